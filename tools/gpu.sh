#!/bin/bash
# The one GPU-box harness (run from the repo root on the GPU box, e.g.
#   gpurun -- 'tools/gpu.sh final r5x').  Every GPU step has its own time limit; the first
# failing step ends the script (no retries).  Output under gpurun_out/, profiles mirrored to
# gpurun_out/profiles/ (profiles/ itself does not travel back).
#
#   tools/gpu.sh tests  <tag> [pytest selection...]      GPU parity tests, one pytest process
#   tools/gpu.sh smoke  <tag>                              __graft_entry__.smoke()
#   tools/gpu.sh bench  <tag> [bench.py args...]           one bench.py line -> gpurun_out/<tag>_bench.json
#   tools/gpu.sh profile <tag> <config> <frames> <streams> [bench args...]
#                                                          rocprofv3 kernel trace + stats, then one PMC
#                                                          pass per counter group -> profiles/<tag>_*
#   tools/gpu.sh ab <tag> "<configs>" <variant>...          same-box A/B: variants alternate within each
#                                                          rep; variant = name:SPEC, SPEC = ENV=VALUE,...,
#                                                          lib=<build dir> (FLACGPU_LIB) or "-"
#                                                          env AB_REPS (2), AB_STEPS (20; 10 for c3-c5),
#                                                          AB_ARGS; rows -> gpurun_out/ab_<tag>.txt
#   tools/gpu.sh stamps <tag>                              phase stamps (build_st: make OUT=build_st
#                                                          EXTRA=-DFG_STAMPS) for C2 and the wide configs
#   tools/gpu.sh diagtests <tag>                           the diagnostic-build-only parity tests (fused, k_ana1,
#                                                          overlapped schedule) against build_diag/libflacgpu.so
#   tools/gpu.sh e2e <tag> <threads...>                    tools/e2e_probe.py once per host MD5 pool size
#                                                          -> gpurun_out/<tag>_e2e_<threads>.json
#   tools/gpu.sh e2etrace <tag>                            rocprofv3 kernel + memory-copy trace of one e2e probe
#                                                          (env E2E_FILES 64, E2E_MANY 0, E2E_THREADS 16) ->
#                                                          tools/overlap.py -> gpurun_out/<tag>_e2e_overlap.json
#   tools/gpu.sh cpuplace <tag>                            CPU-baseline legs alone (no GPU) under each thread
#                                                          placement -> gpurun_out/<tag>_cpu_<place>.json
#   tools/gpu.sh final  <tag>                              tests + smoke + profiles of every config at
#                                                          its bench workload + the default bench line
set -o pipefail
CMD=$1; TAG=${2:-run}; shift 2 || shift $#
REPO=$(pwd)
mkdir -p gpurun_out

summ() {  # one line of a bench JSON (the compact stdout line)
  python3 -c "
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d['value'], d['ms_per_step'], d['output_ok'], json.dumps(d.get('kernel_ms_per_step')))
for k, c in (d.get('configs') or {}).items(): print('  ', k, c['value'], c['ms_per_step'], c['output_ok'], json.dumps(c.get('kernel_ms')))" "$@"
}

do_tests() {
  local sel=${@:-tests}
  timeout -k 10 900 python -u -m pytest $sel -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
  local rc=$?
  tail -3 gpurun_out/${TAG}_pytest.log
  [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/${TAG}_pytest.log | head -30; return $rc; }
}

do_smoke() {
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 ||
    { tail -20 gpurun_out/${TAG}_smoke.log; return 1; }
  tail -1 gpurun_out/${TAG}_smoke.log
}

do_bench() {
  timeout -k 10 600 python -u bench.py "$@" > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err ||
    { tail -20 gpurun_out/${TAG}_bench.err; return 1; }
  cp gpurun_out/bench_detail.json gpurun_out/${TAG}_bench_detail.json 2>/dev/null
  summ gpurun_out/${TAG}_bench.json $TAG
}

do_profile() {  # <ptag> <config> <frames> <streams> [bench args]
  local PT=$1 CFG=$2 FRAMES=$3 STREAMS=$4; shift 4
  local ARGS="--config $CFG --frames $FRAMES --streams $STREAMS --steps 5 --warmup 2 --no-cpu --no-curve --no-e2e --no-sharded --configs= --verify-streams 4 $@"
  local OUT=$REPO/gpurun_out/prof_$PT
  mkdir -p $OUT
  (cd /tmp && export TMPDIR=/tmp &&
   timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 $REPO/bench.py $ARGS > $OUT/kt.log 2>&1) ||
    { echo "kernel trace failed"; tail -5 $OUT/kt.log; return 1; }
  local i=0
  for PMC in "FETCH_SIZE" "WRITE_SIZE" \
             "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
             "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    (cd /tmp && export TMPDIR=/tmp &&
     timeout -s KILL 180 rocprofv3 --pmc $PMC --output-format csv -d $OUT/pmc$i -o pmc -- python3 $REPO/bench.py $ARGS > $OUT/pmc$i.log 2>&1) ||
      { echo "PMC pass $i ($PMC) failed: no further GPU passes"; return 1; }
  done
  local KEY="$CFG:${FRAMES}x${STREAMS}"  # bench.py workload_key
  python3 tools/pmc_summary.py $OUT $PT $FRAMES "$KEY" || return 1
  cp $OUT/kt/kt_kernel_stats.csv profiles/${PT}_kernel_stats.csv
  mkdir -p gpurun_out/profiles && cp profiles/${PT}_* gpurun_out/profiles/
  head -12 profiles/${PT}_summary.md
}

do_ab() {  # "<configs>" <variant>...
  local CFGS=$1; shift
  local SUM=gpurun_out/ab_$TAG.txt REPS=${AB_REPS:-2}
  for cfg in $CFGS; do
    local CA="--configs=" ST=${AB_STEPS:-20}
    if [ "$cfg" != c2 ]; then CA="--config $cfg"; ST=${AB_STEPS:-10}; fi
    for rep in $(seq $REPS); do
      for V in "$@"; do
        local name=${V%%:*} spec=${V#*:} envs=()
        if [ "$spec" != "-" ]; then
          IFS=',' read -ra kv <<< "$spec"
          for a in "${kv[@]}"; do
            case $a in
              lib=*) envs+=("FLACGPU_LIB=$PWD/${a#lib=}/libflacgpu.so") ;;
              *) envs+=("$a") ;;
            esac
          done
        fi
        local out=gpurun_out/ab_${TAG}_${cfg}_${name}_$rep.json
        env "${envs[@]}" timeout -k 10 300 python bench.py $CA --steps $ST --warmup 3 --no-cpu --no-curve \
          --no-e2e --no-sharded --verify-streams 8 $AB_ARGS > $out 2> $out.err || { echo "FAIL $cfg $name"; tail -5 $out.err; return 1; }
        python3 -c "
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(*sys.argv[2:], d['value'], d['ms_per_step'], d['output_ok'], json.dumps(d['kernel_ms_per_step']))" \
          $out $TAG $cfg $name $rep | tee -a $SUM
      done
    done
  done
}

do_stamps() {
  for cfg in "2 16 44100 0" "8 24 96000 0" "2 24 96000 8" "2 32 192000 12"; do
    set -- $cfg
    local t=c${1}_${2}_l$4
    CH=$1 BITS=$2 RATE=$3 LPC=$4 FLACGPU_LIB=$REPO/zig-flac_amd/build_st/libflacgpu.so timeout -k 10 200 \
      python tools/stamps.py > gpurun_out/${TAG}_stamps_$t.log 2>&1 || { echo STAMPS_FAIL $t; tail -20 gpurun_out/${TAG}_stamps_$t.log; return 1; }
    echo "== $t"; grep -v amdgpu.ids gpurun_out/${TAG}_stamps_$t.log
  done
}

do_diagtests() {
  FLACGPU_LIB=$REPO/zig-flac_amd/build_diag/libflacgpu.so timeout -k 10 900 python -u -m pytest tests/test_gpu_fused.py \
    tests/test_gpu_plan.py tests/test_file_host.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "fused or overlapped or one_wave or without_md5" > gpurun_out/${TAG}_diag_pytest.log 2>&1
  local rc=$?
  tail -3 gpurun_out/${TAG}_diag_pytest.log
  return $rc
}

do_e2e() {
  for t in "$@"; do
    FLACGPU_MD5_THREADS=$t timeout -k 10 400 python -u tools/e2e_probe.py --e2e-files ${E2E_FILES:-32,64} \
      --e2e-many ${E2E_MANY:-256} $E2E_ARGS > gpurun_out/${TAG}_e2e_$t.json 2> gpurun_out/${TAG}_e2e_$t.err ||
      { tail -5 gpurun_out/${TAG}_e2e_$t.err; return 1; }
    tail -1 gpurun_out/${TAG}_e2e_$t.json
  done
}

do_e2etrace() {  # rocprofv3 kernel + memory-copy trace (no counters) of one end-to-end probe -> overlap summary
  local OUT=$REPO/gpurun_out/e2etrace_$TAG
  mkdir -p $OUT
  (cd /tmp && export TMPDIR=/tmp && FLACGPU_MD5_THREADS=${E2E_THREADS:-16} timeout -k 10 400 rocprofv3 --kernel-trace \
     --memory-copy-trace --output-format csv -d $OUT/tr -o tr -- python3 $REPO/tools/e2e_probe.py \
     --e2e-files ${E2E_FILES:-64} --e2e-many ${E2E_MANY:-0} $E2E_ARGS > $OUT/tr.log 2>&1) ||
    { echo "trace failed"; tail -5 $OUT/tr.log; return 1; }
  tail -1 $OUT/tr.log
  python3 tools/overlap.py $OUT/tr gpurun_out/${TAG}_e2e_overlap.json > /dev/null
}

do_cpuplace() {
  for place in socket0 idle none; do
    timeout -k 10 300 python -u bench.py --cpu-only --cpu-place $place --configs=c5 > gpurun_out/${TAG}_cpu_$place.json 2> gpurun_out/${TAG}_cpu_$place.err ||
      { tail -5 gpurun_out/${TAG}_cpu_$place.err; return 1; }
    python3 -c "
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for k, v in d['legs'].items():
    print(sys.argv[2], k, v['value'], v['single_core']['value'], v['health'], v['spread']['runs'], v['single_core']['runs'], v['placement'].get('chosen_busy_max'))" gpurun_out/${TAG}_cpu_$place.json $place
  done
}

case $CMD in
  tests) do_tests "$@" ;;
  smoke) do_smoke ;;
  bench) do_bench "$@" ;;
  profile) do_profile "$TAG" "$@" ;;
  ab) do_ab "$@" ;;
  stamps) do_stamps ;;
  cpuplace) do_cpuplace ;;
  e2e) do_e2e "$@" ;;
  e2etrace) do_e2etrace ;;
  diagtests) do_diagtests ;;
  final)
    do_tests && do_smoke &&
    do_profile ${TAG}_c2 c2 262144 16384 > gpurun_out/${TAG}_prof_c2.log 2>&1 &&
    do_profile ${TAG}_c3 c3 65536 16384 > gpurun_out/${TAG}_prof_c3.log 2>&1 &&
    do_profile ${TAG}_c4 c4 65536 16384 > gpurun_out/${TAG}_prof_c4.log 2>&1 &&
    do_profile ${TAG}_c5 c5 65536 16384 > gpurun_out/${TAG}_prof_c5.log 2>&1 &&
    do_bench ;;
  *) sed -n 2,25p "$0"; exit 2 ;;
esac
