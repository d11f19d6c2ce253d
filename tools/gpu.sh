#!/usr/bin/env bash
# One parameterised GPU-box driver (replaces the per-experiment tools/gpu_*.sh scripts).
#
#   gpurun -- bash tools/gpu.sh OUT STEP [STEP ...]
#
# OUT is a directory name under gpurun_out/.  Steps run in order; every GPU step has its own
# time limit, and the script stops at the first failure, time-out, abort or crash.
#   tests               pytest -m gpu (one process)
#   pytest:NAME:ARGS    pytest -m gpu ARGS (test files / -k filters) -> OUT/pytest_NAME.log
#   smoke               __graft_entry__.smoke()
#   bench:NAME[:ARGS]   python bench.py ARGS  -> OUT/NAME.json  (ARGS: comma-separated flags)
#   prof:NAME[:ARGS]    rocprofv3 --kernel-trace --stats around bench.py ARGS -> OUT/prof_NAME/
#   pmc:NAME:CTRS[:ARGS] rocprofv3 --pmc CTRS (comma list) around bench.py ARGS -> OUT/pmc_NAME/
#   py:NAME:SCRIPT[:ARGS] python SCRIPT ARGS -> OUT/NAME.log
#   pyprof:NAME:SCRIPT[:ARGS] the same under rocprofv3 --kernel-trace --stats -> OUT/prof_NAME/
#   pypmc:NAME:CTRS:SCRIPT[:ARGS] the same under rocprofv3 --pmc CTRS -> OUT/pmc_NAME/
#   env:VAR=VALUE       export VAR=VALUE for the following steps (env:VAR= unsets it)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:?usage: gpu.sh OUT STEP...}
shift
mkdir -p "$OUT"

fail() { echo "FAILED: $*" | tee -a "$OUT/status.txt"; exit 1; }
args_of() { echo "${1//,/ }"; }

for step in "$@"; do
    kind=${step%%:*}
    rest=${step#*:}
    [ "$rest" = "$step" ] && rest=""
    name=${rest%%:*}
    extra=""
    [ "$rest" != "$name" ] && extra=${rest#*:}
    echo "[$(date +%T)] $step" | tee -a "$OUT/status.txt"
    case $kind in
        tests)
            timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread \
                > "$OUT/pytest_gpu.log" 2>&1 || fail "pytest rc=$?" ;;
        pytest)
            # shellcheck disable=SC2046
            timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 240 --timeout-method thread $(args_of "$extra") \
                > "$OUT/pytest_$name.log" 2>&1 || fail "pytest $name rc=$?" ;;
        smoke)
            timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
                || fail "smoke rc=$?" ;;
        bench)
            # shellcheck disable=SC2046
            timeout -k 10 400 python bench.py $(args_of "$extra") --json-out "$OUT/$name.json" \
                > "$OUT/$name.log" 2>&1 || fail "bench $name rc=$?" ;;
        prof)
            # shellcheck disable=SC2046
            timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$name" -o run \
                -- python3 bench.py $(args_of "$extra") > "$OUT/prof_$name.log" 2>&1 || fail "prof $name rc=$?" ;;
        pmc)
            ctrs=${extra%%:*}
            bargs=""
            [ "$extra" != "$ctrs" ] && bargs=${extra#*:}
            # shellcheck disable=SC2046
            timeout -s KILL 120 rocprofv3 --pmc $(args_of "$ctrs") --output-format csv -d "$OUT/pmc_$name" -o run \
                -- python3 bench.py $(args_of "$bargs") > "$OUT/pmc_$name.log" 2>&1 || fail "pmc $name rc=$?" ;;
        pyprof)
            script=${extra%%:*}
            pargs=""
            [ "$extra" != "$script" ] && pargs=${extra#*:}
            # shellcheck disable=SC2046
            timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$name" -o run \
                -- python3 -u "$script" $(args_of "$pargs") > "$OUT/prof_$name.log" 2>&1 || fail "pyprof $name rc=$?" ;;
        pypmc)
            ctrs=${extra%%:*}
            rest2=${extra#*:}
            script=${rest2%%:*}
            pargs=""
            [ "$rest2" != "$script" ] && pargs=${rest2#*:}
            # shellcheck disable=SC2046
            timeout -s KILL 120 rocprofv3 --pmc $(args_of "$ctrs") --output-format csv -d "$OUT/pmc_$name" -o run \
                -- python3 -u "$script" $(args_of "$pargs") > "$OUT/pmc_$name.log" 2>&1 || fail "pypmc $name rc=$?" ;;
        py)
            script=${extra%%:*}
            pargs=""
            [ "$extra" != "$script" ] && pargs=${extra#*:}
            # shellcheck disable=SC2046
            timeout -k 10 600 python -u "$script" $(args_of "$pargs") > "$OUT/$name.log" 2>&1 \
                || fail "py $name rc=$?" ;;
        env)
            var=${rest%%=*}
            val=${rest#*=}
            if [ -n "$val" ]; then export "$var=$val"; else unset "$var"; fi ;;
        *) fail "unknown step $step" ;;
    esac
done
echo "[$(date +%T)] done" | tee -a "$OUT/status.txt"
