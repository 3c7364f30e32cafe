#!/bin/bash
# Host facts of the GPU box (CPU model, cores per socket, CPU share) + MD5 rate of one core.
mkdir -p gpurun_out
{
lscpu
echo "nproc=$(nproc)"
cat /sys/fs/cgroup/cpu.max 2>/dev/null
python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))"
command -v zig || echo "zig: absent"
python3 - <<'PY'
import hashlib, time, os
b = os.urandom(256 << 20)
t = time.perf_counter(); hashlib.md5(b).digest(); dt = time.perf_counter() - t
print(f"hashlib md5 one core: {len(b)/dt/1e6:.0f} MB/s")
PY
} > gpurun_out/probe_host.txt 2>&1
