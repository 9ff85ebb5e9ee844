#!/bin/bash
# One launcher for the GPU box (replaces round 3's one-shot scripts/r3/gpu_round3*.sh):
#   gpurun --timeout T -- 'bash scripts/gpu_steps.sh OUTDIR STEP [STEP ...]'
# Every step runs under its own time limit, writes under gpurun_out/OUTDIR, and the first failing step ends the call
# (no retries).  Steps:
#   tests            the whole -m gpu suite
#   tests:EXPR       -m gpu tests selected by pytest -k EXPR
#   smoke            __graft_entry__.smoke()
#   bench            python bench.py (defaults) -> bench.json
#   bench20          python bench.py --steps 20 --warmup 5 -> bench_k20.json
#   prof             rocprofv3 --kernel-trace --stats of bench.py --steps 20
#   multistart:RUNS  scripts/msk_multistart_probe.py --native --runs RUNS (e.g. 64:0.1,512:0.1)
#   specms:RUNS:SOFT the same with the BatchedIpm specification and soft_resto_pderror_reduction_factor SOFT
#   py:SCRIPT[:ARGS] python SCRIPT ARGS (ARGS with commas for spaces), stdout to SCRIPT's name .txt
#   bin:PATH[:ARGS]  a binary built here (e.g. scripts/micro/bin/colloc_bw), stdout to its name .txt
#   env:NAME=VALUE   export NAME=VALUE for the steps after it (e.g. env:CFX_LIB=cocofest_amd/libcfx_recip.so)
#   limit:SECONDS    time limit of the py: steps after it (default 900)
#   trace:SCRIPT[:ARGS]  rocprofv3 --kernel-trace --stats (CSV) over python3 SCRIPT ARGS -> trace_<script>/
#   pmc:CTRS[@LABEL]:SCRIPT[:ARGS]  rocprofv3 --pmc CTRS ('+'-separated, one pass; FETCH_SIZE and WRITE_SIZE each
#                    alone) over python3 SCRIPT ARGS -> pmc_[LABEL_]<first counter>/
set -o pipefail
out=gpurun_out/$1
shift
mkdir -p "$out"
export TMPDIR=/tmp
run() {  # run LIMIT LOGNAME CMD...
    local lim=$1 log=$2
    shift 2
    echo "== $(date +%T) $log: $*"
    timeout -k 10 "$lim" "$@" > "$out/$log" 2>&1
    local rc=$?
    tail -n 5 "$out/$log"
    if [ $rc -ne 0 ]; then
        echo "== step $log failed: rc $rc"
        exit $rc
    fi
}
pylim=900
for step in "$@"; do
    case "$step" in
        tests) run 600 pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ;;
        tests:*) run 600 "pytest_${step#tests:}.log" python -u -m pytest tests -m gpu -x -v --timeout 300 \
                     --timeout-method thread -k "${step#tests:}" ;;
        smoke) run 300 smoke.log python -c "import __graft_entry__ as g; g.smoke()" ;;
        bench) run 600 bench.log python bench.py && grep '^{' "$out/bench.log" | tail -n 1 > "$out/bench.json" ;;
        bench20) run 600 bench20.log python bench.py --steps 20 --warmup 5 &&
                 grep '^{' "$out/bench20.log" | tail -n 1 > "$out/bench_k20.json" ;;
        prof) run 900 prof.log rocprofv3 --kernel-trace --stats -d "$out/prof" -o run -- python3 bench.py --steps 20 ;;
        multistart:*) run 1100 "multistart_${step#multistart:}.log" python3 -u scripts/msk_multistart_probe.py --native \
                          --runs "${step#multistart:}" --jsonl "$out/multistart.jsonl" ;;
        specms:*) r=${step#specms:}
                  run 1100 "specms_${r}.log" python3 -u scripts/msk_multistart_probe.py --runs "${r%:*}" \
                      --soft "${r##*:}" --jsonl "$out/specms.jsonl" ;;
        py:*) spec=${step#py:}
              script=${spec%%:*}
              args=""
              [ "$spec" != "$script" ] && args=${spec#*:}
              # shellcheck disable=SC2086
              run "$pylim" "$(basename "$script" .py).txt" python3 -u "$script" ${args//,/ } ;;
        bin:*) spec=${step#bin:}
               exe=${spec%%:*}
               args=""
               [ "$spec" != "$exe" ] && args=${spec#*:}
               # shellcheck disable=SC2086
               run 300 "$(basename "$exe").txt" "$exe" ${args//,/ } ;;
        pmc:*) spec=${step#pmc:}
               ctr=${spec%%:*}
               rest=${spec#*:}
               script=${rest%%:*}
               args=""
               [ "$rest" != "$script" ] && args=${rest#*:}
               # shellcheck disable=SC2086
               tag=${ctr%%+*}
               if [[ "$ctr" == *@* ]]; then tag="${ctr#*@}_${tag%%@*}"; ctr=${ctr%%@*}; fi
               # shellcheck disable=SC2086
               run 180 "pmc_${tag}.log" timeout -s KILL 150 rocprofv3 --pmc ${ctr//+/ } -d "$out/pmc_${tag}" -o run -- \
                   python3 "$script" ${args//,/ } ;;
        limit:*) pylim=${step#limit:} ;;
        trace:*) spec=${step#trace:}
                 script=${spec%%:*}
                 args=""
                 [ "$spec" != "$script" ] && args=${spec#*:}
                 name=$(basename "$script" .py)
                 # shellcheck disable=SC2086
                 run "$pylim" "trace_${name}.log" rocprofv3 --kernel-trace --stats --output-format csv \
                     -d "$out/trace_${name}" -o run -- python3 -u "$script" ${args//,/ } ;;
        env:*) kv=${step#env:}
               export "${kv%%=*}=${kv#*=}"
               echo "== export ${kv%%=*}=${kv#*=}" ;;
        *) echo "unknown step $step"; exit 2 ;;
    esac
done
echo "== $(date +%T) all steps done"
