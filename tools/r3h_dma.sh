#!/bin/bash
# r3h: LDS-DMA hidden from the wait-count pass, k_pack4 descriptors by LDS-DMA a frame ahead,
# tickets behind the stores, LDS-only barriers in k_pack: GPU suite, then same-box A/B vs r3f.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3h_pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/r3h_pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r3h_pytest_gpu.log | head; exit $rc; }
bash tools/ab_cfgs.sh r3h "c2 c4 c3 c5" zig-flac_amd/build_crc zig-flac_amd/build || exit 1
