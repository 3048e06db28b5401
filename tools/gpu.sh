#!/bin/bash
# The GPU-box measurement script (run through gpurun from the repo root).  Subcommands, each run under its own
# time limit, chained with && so that the first failure ends the call:
#
#   tools/gpu.sh tests [pytest paths / -k expr ...]  the -m gpu suite (or a selection)    -> $O/gpu_tests.log
#   tools/gpu.sh bench [bench.py args ...]           one bench line                        -> $O/bench.json
#   tools/gpu.sh prof [bench.py args ...]            the bench under rocprofv3 --stats     -> $O/prof/, $O/bench_prof.json
#   tools/gpu.sh pmc  [bench.py args ...]            FETCH_SIZE / WRITE_SIZE passes (separate runs) summarised by
#                                                    tools/pmc_summary.py, copied to profiles/pmc_$T_$NAME.json
#   tools/gpu.sh sq   [bench.py args ...]            one SQ instruction-counter pass       -> $O/sq/
#   tools/gpu.sh ab name1[:ENV=V] name2 ...          A/B of engine builds (tools/build_variants.sh) on the bench
#   tools/gpu.sh cfgprof name [bench.py args ...]    one BASELINE config sub-line (w7_100_shells, nebular_onezone,
#                                                    kilonova) under rocprofv3 --stats -> $O/cfg_$name/, $O/cfg_$name.json
#   tools/gpu.sh pcs  [bench.py args ...]            stochastic PC sampling (cycles) of a short bench run -> $O/pcs/
#   tools/gpu.sh stamps name [bench.py args ...]     the cycle-stamp build (build/ab/stamps, -DARTIS_STAMPS) with
#                                                    ARTIS_GPU_STATS=1 on a bench run -> $O/stamps_$name.{json,err}
#   tools/gpu.sh pre name1[:ENV=V] name2 ...         the precompute alone (tools/precompute_ab.py) per engine build,
#                                                    under rocprofv3 --stats -> $O/pre_<name>.{json,txt}
#   tools/gpu.sh sqpy name script.py [args]          one SQ instruction-counter pass over a python script -> $O/sq_<name>.txt
#   tools/gpu.sh final                               tests, prof, pmc, default bench line (the round-end set)
#
# Environment: T (tag, default "r4"), O (output dir, default gpurun_out/$T), NAME (pmc summary name, default
# "bench"), P (packets for pmc / sq / ab, default 1e7), BENCH_ARGS (extra bench args for ab), ENVS (env for ab).
cd /root/repo || exit 1
export TMPDIR=/tmp
T=${T:-r5}
O=${O:-gpurun_out/$T}
mkdir -p "$O"
cmd=$1
shift

run_tests() {
  local args=("$@")
  [ ${#args[@]} -eq 0 ] && args=(tests)
  timeout -k 10 900 python -u -m pytest "${args[@]}" -m gpu -x -v --timeout 300 --timeout-method thread \
    > "$O/gpu_tests.log" 2>&1
  local rc=$?
  tail -1 "$O/gpu_tests.log"
  return $rc
}

run_bench() {
  timeout -k 10 900 python3 -u bench.py "$@" > "$O/bench.json" 2> "$O/bench.err" && tail -c 400 "$O/bench.json"
}

# (the rocpd database is summarised into $O/kernel_stats.csv and removed: gpurun merges at most 64 MiB back)
run_prof() {
  rm -rf "$O/prof"
  timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run -- python3 -u bench.py --no-cpu-baseline "$@" \
    > "$O/bench_prof.json" 2> "$O/bench_prof.err" &&
  python3 tools/rocpd_stats.py "$O/prof/run_results.db" --csv "$O/kernel_stats.csv" && rm -rf "$O/prof"
}

run_cfgprof() {
  local name=$1
  shift
  rm -rf "$O/cfg_$name"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/cfg_$name" -o run -- python3 -u bench.py \
    --baseline-config "$name" "$@" > "$O/cfg_$name.json" 2> "$O/cfg_$name.err" && tail -c 300 "$O/cfg_$name.json"
}

# pmc [bench args]: the bench's defaults are --packets 1e7 --nts 10; the summary needs the same numbers
run_pmc() {
  local name=${NAME:-bench} packets=${P:-10000000} nts=10 vp=0 a
  local args=("$@")
  for ((i = 0; i < ${#args[@]}; i++)); do
    a=${args[$i]}
    case "$a" in
      --packets) packets=${args[$((i + 1))]} ;;
      --nts) nts=${args[$((i + 1))]} ;;
      --vpkt) vp=${args[$((i + 1))]} ;;
    esac
  done
  # (argparse keeps the last --packets, the one parsed above)
  local B="python3 bench.py --packets $packets --steps 1 --warmup 0 --no-cpu-baseline --no-update-grid --no-extra $*"
  mkdir -p "$O/pmc_$name"
  rm -rf "$O/pmc_$name/fetch" "$O/pmc_$name/write"
  timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$O/pmc_$name/fetch" -o run -- $B > "$O/pmc_$name/f.log" 2>&1 &&
  timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$O/pmc_$name/write" -o run -- $B > "$O/pmc_$name/w.log" 2>&1 &&
  python3 tools/pmc_summary.py --fetch "$O/pmc_$name/fetch" --write "$O/pmc_$name/write" --packets "$packets" --ngrid 50 \
    --nts "$nts" $([ "$vp" != 0 ] && echo --vpkt "$vp") --out "$O/pmc_$name.json" &&
  cp "$O/pmc_$name.json" "profiles/pmc_${T}_$name.json" && rm -rf "$O/pmc_$name/fetch" "$O/pmc_$name/write"
}

run_sq() {
  rm -rf "$O/sq"
  mkdir -p "$O/sq"
  timeout -s KILL 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VALU \
    SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM --kernel-trace -d "$O/sq/db" -o run -- python3 bench.py \
    --packets ${P:-2000000} --steps 1 --warmup 0 --no-cpu-baseline --no-update-grid --no-extra "$@" > "$O/sq/sq.log" 2>&1
}

# sqpy name script.py [args]: one SQ counter pass over any python script (e.g. tools/precompute_ab.py)
run_sqpy() {
  local name=$1
  shift
  rm -rf "$O/sq_$name"
  mkdir -p "$O/sq_$name"
  timeout -s KILL 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VALU \
    SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM --kernel-trace -d "$O/sq_$name/db" -o run -- python3 "$@" \
    > "$O/sq_$name/run.log" 2>&1 && python3 tools/sq_summary.py "$O/sq_$name/db" | tee "$O/sq_$name.txt"
}

run_stamps() {
  local name=$1
  shift
  ARTIS_GPU_SO=${STAMPS_SO:-build/ab/stamps/libartis_gpu.so} ARTIS_GPU_STATS=1 timeout -k 10 600 python3 -u bench.py --no-cpu-baseline \
    --no-update-grid --no-extra "$@" > "$O/stamps_$name.json" 2> "$O/stamps_$name.err" && grep "artis_gpu\]" "$O/stamps_$name.err" | tail -12
}

run_pcs() {
  rm -rf "$O/pcs"
  mkdir -p "$O/pcs"
  timeout -s KILL 120 rocprofv3 -L > "$O/pcs/list.txt" 2>&1
  timeout -s KILL 400 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles \
    --pc-sampling-interval ${PCS_INTERVAL:-1048576} --output-format csv -d "$O/pcs/db" -o run -- python3 bench.py \
    --packets ${P:-2000000} --steps 1 --warmup 0 --no-cpu-baseline --no-update-grid --no-extra "$@" > "$O/pcs/pcs.log" 2>&1
}

run_ab() {
  local v name envs so tag
  for v in "$@"; do
    name=${v%%:*}; envs=""; [[ "$v" == *:* ]] && envs=${v#*:}
    so=build/ab/$name/libartis_gpu.so; [ "$name" = main ] && so=artis_amd/lib/libartis_gpu.so
    tag=$(echo "$v" | tr -c 'A-Za-z0-9_\n' '_')
    env ARTIS_GPU_SO=$so $ENVS $envs timeout -k 10 400 python3 bench.py --packets ${P:-10000000} --steps 1 --warmup 1 \
      --no-cpu-baseline --no-update-grid --no-extra $BENCH_ARGS > "$O/ab_$tag.json" 2> "$O/ab_$tag.err" ||
      { echo "FAIL $v"; tail -5 "$O/ab_$tag.err"; return 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'value', round(d['value']), 'ms', round(d['ms_per_step']), 'precompute', round(d.get('precompute_ms', 0)), {k: round(x) for k, x in d['kernel_ms'].items()}, 'frac', round(d['roofline']['frac'], 4))" "$O/ab_$tag.json" "$v"
  done
}

run_pre() {
  local v name envs so tag db
  for v in "$@"; do
    name=${v%%:*}; envs=""; [[ "$v" == *:* ]] && envs=${v#*:}
    so=build/ab/$name/libartis_gpu.so; [ "$name" = main ] && so=artis_amd/lib/libartis_gpu.so
    tag=$(echo "$v" | tr -c 'A-Za-z0-9_\n' '_')
    rm -rf "$O/pre_$tag"
    env ARTIS_GPU_SO=$so $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/pre_$tag" -o run -- python3 -u \
      tools/precompute_ab.py > "$O/pre_$tag.json" 2> "$O/pre_$tag.err" || { echo "FAIL $v"; tail -5 "$O/pre_$tag.err"; return 1; }
    db=$O/pre_$tag/run_results.db
    { echo "$v $(tail -c 200 "$O/pre_$tag.json")"; python3 tools/kstat_short.py "$db" 12; } | tee "$O/pre_$tag.txt"
  done
}

case "$cmd" in
  tests) run_tests "$@" ;;
  bench) run_bench "$@" ;;
  prof) run_prof "$@" ;;
  pmc) run_pmc "$@" ;;
  sq) run_sq "$@" ;;
  ab) run_ab "$@" ;;
  cfgprof) run_cfgprof "$@" ;;
  pcs) run_pcs "$@" ;;
  stamps) run_stamps "$@" ;;
  pre) run_pre "$@" ;;
  sqpy) run_sqpy "$@" ;;
  final) run_tests && run_prof --no-extra && run_pmc && run_bench ;;
  *) echo "usage: tools/gpu.sh tests|bench|prof|pmc|sq|ab|final [args]"; exit 2 ;;
esac
