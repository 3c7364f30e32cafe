"""Golden vectors (tests/golden/, made by tests/golden/make_golden.py).

CPU: the restatement reproduces every committed vector byte for byte, and the
synthetic input generator still produces the committed inputs.
GPU: libflacgpu.so produces the same bytes, frame sizes and MD5.
"""
import hashlib
import json
import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
sys.path.insert(0, GOLD)

import make_golden  # noqa: E402
import oracle_ref  # noqa: E402

MANIFEST = json.load(open(os.path.join(GOLD, "manifest.json")))["cases"]
IDS = [c["name"] for c in MANIFEST]


def _inputs(c):
    pcm = make_golden.make_pcm(c["name"], c["channels"], c["bits"], c["rate"], c["n_samples"], c["stream_seed"])
    assert hashlib.sha256(pcm).hexdigest() == c["pcm_sha256"], "synthetic input generator drifted"
    gold = open(os.path.join(GOLD, c["name"] + ".flac"), "rb").read()
    assert hashlib.sha256(gold).hexdigest() == c["out_sha256"]
    return pcm, gold


@pytest.mark.parametrize("c", MANIFEST, ids=IDS)
def test_oracle_reproduces_golden(c):
    pcm, gold = _inputs(c)
    if c["kind"] == "file":
        out = oracle_ref.encode_file(pcm, c["channels"], c["bits"], c["rate"], c["block"])
        assert out == gold
    else:
        out, sizes, md5 = oracle_ref.encode_stream(pcm, c["channels"], c["bits"], c["rate"], c["block"],
                                                   first_frame=c["first_frame"])
        assert out == gold and sizes == c["frame_bytes"] and md5.hex() == c["md5"]


@pytest.mark.gpu
@pytest.mark.parametrize("c", MANIFEST, ids=IDS)
def test_gpu_reproduces_golden(c):
    import flacgpu

    pcm, gold = _inputs(c)
    with flacgpu.Encoder(c["channels"], c["bits"], c["rate"], max_frames=64, block_size=c["block"]) as enc:
        out, sizes = enc.encode_frames(pcm, first_frame=c["first_frame"])
        md5 = enc.md5(pcm)
    if c["kind"] == "file":
        gold = gold[73:]  # frames after fLaC + STREAMINFO + VORBIS_COMMENT
    else:
        assert list(sizes) == c["frame_bytes"]
    assert out == gold
    assert md5.hex() == c["md5"]
