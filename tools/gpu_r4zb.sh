#!/bin/bash
# r4zb: streaming (nontemporal) frame stores in the pack kernels, C2 only (build_x: fg_enc_b2_l0 with
# -DFG_STORE_NT=1, everything else HEAD): GPU suite on it, then the same-box A/B
set -o pipefail
mkdir -p gpurun_out
FLACGPU_LIB=$PWD/zig-flac_amd/build_x/libflacgpu.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4zb_pytest.log 2>&1 || { tail -30 gpurun_out/r4zb_pytest.log; exit 1; }
tail -2 gpurun_out/r4zb_pytest.log
AB_REPS=3 tools/ab.sh r4zb "c2" base:- nt:lib=zig-flac_amd/build_x
