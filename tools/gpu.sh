#!/bin/bash
# tools/gpu.sh TAG STEP [STEP ...] -- the one GPU-box runner.
#
#   gpurun --timeout 900 -- bash tools/gpu.sh r02a test bench trace:--steps,5
#
# Every step runs under its own time limit; the first failure ends the call
# (set -e), so nothing touches the GPU after a fault, abort or timeout.
# Outputs go to gpurun_out/TAG/<n>_<step>.{json,log,...}.  ARGS are
# comma-separated (commas become spaces).
#
#   test[:PATH]          pytest -m gpu (all of tests/, or PATH)
#   smoke                __graft_entry__.smoke()
#   bench[:ARGS]         python bench.py ARGS            (stdout = the JSON line)
#   trace[:ARGS]         rocprofv3 --kernel-trace --stats -- python bench.py ARGS
#   pmc:CTRS[:ARGS]      rocprofv3 --pmc CTRS (+ kernel trace) -- python bench.py ARGS
#                        (CTRS '+'-separated; one pass, within the per-block limits)
#   pmcpy:CTRS:SCRIPT[:ARGS]  rocprofv3 --pmc CTRS -- python SCRIPT ARGS (one pass)
#   calib                FETCH_SIZE / WRITE_SIZE passes over tools/calib_fetch
#   py:SCRIPT[:ARGS]     python SCRIPT ARGS              (probes under tools/; limit
#                        $PY_TIMEOUT s, default 600 -- set it with env:PY_TIMEOUT=N)
#   dist:N[:ARGS]        torch.distributed.run N gloo ranks on this one GPU:
#                        python bench.py --gpus N --backend gloo ARGS
#   env:VAR=VAL          export VAR=VAL for the following steps (VAL empty: unset)
#   counters             rocprofv3 -L (the counters this GPU offers) -> NN_counters.txt
set -e
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
n=0
for step in "$@"; do
    n=$((n + 1))
    kind=${step%%:*}
    rest=""
    [[ "$step" == *:* ]] && rest=${step#*:}
    args=${rest//,/ }
    p="$O/$(printf %02d $n)_$kind"
    # bench.py writes its library map here at exit (record_maps_at_exit): kept
    # only when the step fails, so a fault's PCs can be matched to a library
    export MF_MAPS_DIR="$p.maps"
    echo "[gpu.sh $(date +%H:%M:%S)] step $n: $step"
    case $kind in
    test)
        timeout -k 10 900 python -u -m pytest ${args:-tests} -m gpu -x -v --timeout 240 \
            --timeout-method thread > "$p.log" 2>&1 ;;
    smoke)
        timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$p.log" 2>&1 ;;
    bench)
        timeout -k 10 600 python -u bench.py $args > "$p.json" 2> "$p.log" ;;
    trace)
        timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$p" -o run \
            -- python "$R/bench.py" $args > "$p.json" 2> "$p.log" ;;
    pmc)
        ctrs=${rest%%:*}
        bargs=""
        [[ "$rest" == *:* ]] && bargs=${rest#*:}
        timeout -s KILL 300 rocprofv3 --pmc ${ctrs//+/ } --kernel-trace --output-format csv -d "$p" \
            -o run -- python "$R/bench.py" ${bargs//,/ } > "$p.json" 2> "$p.log" ;;
    pmcpy)
        # pmcpy:CTRS:SCRIPT[:ARGS] -- one PMC pass over a probe script
        ctrs=${rest%%:*}
        srest=${rest#*:}
        script=${srest%%:*}
        sargs=""
        [[ "$srest" == *:* ]] && sargs=${srest#*:}
        timeout -s KILL 300 rocprofv3 --pmc ${ctrs//+/ } --kernel-trace --output-format csv -d "$p" \
            -o run -- python "$R/$script" ${sargs//,/ } > "$p.out" 2> "$p.log" ;;
    calib)
        timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv \
            -d "${p}_fetch" -o run -- "$R/tools/calib_fetch" > "${p}_fetch.log" 2>&1
        timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv \
            -d "${p}_write" -o run -- "$R/tools/calib_fetch" > "${p}_write.log" 2>&1 ;;
    py)
        script=${rest%%:*}
        pargs=""
        [[ "$rest" == *:* ]] && pargs=${rest#*:}
        timeout -k 10 ${PY_TIMEOUT:-600} python -u "$script" ${pargs//,/ } > "$p.out" 2> "$p.log" ;;
    dist)
        nr=${rest%%:*}
        dargs=""
        [[ "$rest" == *:* ]] && dargs=${rest#*:}
        timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$nr" \
            --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus "$nr" --backend gloo \
            ${dargs//,/ } > "$p.json" 2> "$p.log" ;;
    counters)
        timeout -k 10 120 rocprofv3 -L > "$p.txt" 2>&1 ;;
    env)
        var=${rest%%=*}; val=${rest#*=}
        if [ -z "$val" ]; then unset "$var"; else export "$var=$val"; fi ;;
    *)
        echo "unknown step $step" >&2; exit 2 ;;
    esac
    rm -rf "$p.maps"          # reached only when the step exited 0 (set -e)
done
echo "[gpu.sh $(date +%H:%M:%S)] done"
