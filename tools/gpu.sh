#!/bin/bash
# GPU-box recipe runner (gpurun): one script with named steps instead of one-off files.
#   bash tools/gpu.sh <out-dir-name> <step> [<step> ...]
# Every step runs under its own timeout and writes its log under gpurun_out/<out-dir-name>/;
# the first failing step ends the script (nothing more touches the GPU after a failure).
# Steps:
#   tests           the whole -m gpu suite, one process, per-test timeout
#   tests:<expr>    the -m gpu tests matching -k <expr>
#   testsall        the whole -m gpu suite without -x (every failure listed; a GPU fault still ends it)
#   smoke           __graft_entry__.smoke()
#   bench           the default bench line (driver form: python bench.py)
#   bench:<args>    bench.py with extra arguments (commas for spaces: bench:--workload,c1)
#   torchrun:<N>:<args>  bench.py --gpus N under torchrun (N ranks; --rehearse shares the box's GPU)
#   prof            rocprofv3 kernel trace + PMC passes of a short C2 bench (tools/profile.sh)
#   prof:<args>     the same over bench.py <args> (commas for spaces)
#   segv            the round-3 traced 8-caller percall_bench (kernel + memory-copy trace) with the
#                   fault handler armed (PERCALL_SEGV_LOG): one run, diagnostics kept if it faults
#   percall:<args>  percall_bench <args> (commas for spaces), untraced
#   ab:<lib>        same-box A/B: C2 line with lib/<lib> (base) vs the in-tree library, x3 alternating
#   hptrace[:chunk] kernel + copy trace and per-chunk host timeline of 1M-pair host-buffer calls
#   hpapi[:chunk]   the same plus the HIP runtime API trace
#   export:VAR=VAL  set an environment variable for the following steps (unset:VAR clears it)
#   py:<file>       python -u <file> (a probe script under tools/)
# (rounds 1-3 kept one file per gpurun call, tools/gpu_*.sh; they are in git history, baea391)
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
name=${1:?out dir name}; shift
O=gpurun_out/$name
mkdir -p "$O"
export TMPDIR=/tmp
fail() { echo "step $1 FAILED (rc $2); log tail:"; tail -30 "$3"; exit 1; }
sp() { echo "${1//,/ }"; }
n=0
for step in "$@"; do
    n=$((n + 1))
    kind=${step%%:*}; arg=""; [[ "$step" == *:* ]] && arg=${step#*:}
    t0=$(date +%s)
    case "$kind" in
    tests)
        log=$O/gpu_tests${arg:+_$arg}.log
        k=(); [ -n "$arg" ] && k=(-k "$arg")
        timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "${k[@]}" \
            > "$log" 2>&1 || fail "$step" $? "$log"
        tail -1 "$log" ;;
    testsall)
        log=$O/gpu_tests_all.log
        timeout -k 10 1100 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
            > "$log" 2>&1 || fail "$step" $? "$log"
        tail -1 "$log" ;;
    smoke)
        log=$O/smoke.log
        timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$log" 2>&1 || fail "$step" $? "$log"
        tail -3 "$log" ;;
    bench)
        log=$O/bench${arg:+_$(echo "$arg" | tr -c 'A-Za-z0-9\n' '_' | cut -c1-60)}_$n.log
        timeout -k 10 600 python bench.py $(sp "$arg") > "$log" 2>&1 || fail "$step" $? "$log"
        tail -1 "$log" | cut -c1-1500 ;;
    torchrun)
        nr=${arg%%:*}; targs=${arg#*:}
        log=$O/torchrun_${nr}_$n.log
        timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$nr" --master-addr 127.0.0.1 \
            --master-port $((29000 + n)) bench.py --gpus "$nr" $(sp "$targs") > "$log" 2>&1 || fail "$step" $? "$log"
        grep '^{' "$log" | tail -1 | cut -c1-1500 ;;
    prof)
        OUT=$O/prof${arg:+_$(echo "$arg" | tr -c 'A-Za-z0-9\n' '_' | cut -c1-40)} \
            ARGS="${arg:+$(sp "$arg") }--steps 5 --warmup 1 --no-cpu --no-host-path" \
            timeout -k 10 1100 bash tools/profile.sh > "$O/prof.log" 2>&1 || fail "$step" $? "$O/prof.log"
        tail -1 "$O/prof.log" ;;
    segv)
        log=$O/segv_trace.log
        rm -rf "$O/segv_trace"
        PERCALL_SEGV_LOG=$O/segv_diag.txt PERCALL_MAPS_LOG=$O/segv_maps.txt timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace \
            --output-format csv -d "$O/segv_trace" -- bwa-mem2-arm_amd/lib/percall_bench 200000 8 1000 \
            > "$log" 2>&1; rc=$?
        [ -f "$O/segv_diag.txt" ] && { echo "FAULT diagnostics:"; head -40 "$O/segv_diag.txt"; }
        [ $rc -eq 0 ] || fail "$step" $rc "$log"
        grep '^{' "$log" | cut -c1-600 ;;
    percall)
        log=$O/percall_$n.log
        timeout -k 10 300 bwa-mem2-arm_amd/lib/percall_bench $(sp "$arg") > "$log" 2>&1 || fail "$step" $? "$log"
        tail -1 "$log" | cut -c1-1500 ;;
    ab)
        # same-box A/B of the in-tree library (new) against lib/<arg> (base): C2 bench lines
        # alternating base / new three times, value and DP kernel ms of each
        log=$O/ab_$arg.log; : > "$log"
        for k in 1 2 3; do
            for v in base new; do
                if [ $v = base ]; then L=$PWD/bwa-mem2-arm_amd/lib/$arg; else L=$PWD/bwa-mem2-arm_amd/lib/libbsw_hip.so; fi
                BSW_HIP_LIB=$L timeout -k 10 200 python bench.py --no-cpu --no-host-path --steps 30 --warmup 3 \
                    > "$O/ab_run.log" 2>&1 || fail "$step" $? "$O/ab_run.log"
                python3 -c "import json;d=json.loads(open('$O/ab_run.log').read().strip().splitlines()[-1]);print('$v', d['value'], d['roofline']['launch_ms'])" | tee -a "$log"
            done
        done ;;
    abhp)
        # same-box A/B of the drop-in host path: tools/host_path_once.py (1M-pair calls after a
        # device warm-up) with lib/<arg> (base) vs the in-tree library (new), alternating x3;
        # per run the median of calls 3..8
        log=$O/abhp_$arg.log; : > "$log"
        for k in 1 2 3; do
            for v in base new; do
                if [ $v = base ]; then L=$PWD/bwa-mem2-arm_amd/lib/$arg; else L=$PWD/bwa-mem2-arm_amd/lib/libbsw_hip.so; fi
                BSW_HIP_LIB=$L timeout -k 10 200 python tools/host_path_once.py 196608 8 1 > "$O/abhp_run.log" 2>&1 \
                    || fail "$step" $? "$O/abhp_run.log"
                python3 -c "import statistics as S;v=[float(l.split()[1]) for l in open('$O/abhp_run.log') if l.startswith('call')][2:];print('$v', round(S.median(v),3), v)" | tee -a "$log"
            done
        done ;;
    hptrace)
        # the drop-in host path's timeline: per-chunk host times (BSW_DEBUG_HP) and a kernel +
        # copy trace of a few 1M-pair bsw_get_scores calls (tools/host_path_once.py [chunk] [calls])
        rm -rf "$O/hptrace"
        BSW_DEBUG_HP=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
            -d "$O/hptrace" -- python3 tools/host_path_once.py ${arg:-262144} 4 > "$O/hptrace.log" 2>&1 \
            || fail "$step" $? "$O/hptrace.log"
        grep '^call' "$O/hptrace.log" ;;
    hpapi)
        # hptrace plus the HIP runtime API trace (per-thread host timeline of every runtime call)
        rm -rf "$O/hpapi"
        BSW_DEBUG_HP=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv \
            -d "$O/hpapi" -- python3 tools/host_path_once.py ${arg:-262144} 4 > "$O/hpapi.log" 2>&1 \
            || fail "$step" $? "$O/hpapi.log"
        grep '^call' "$O/hpapi.log" ;;
    export)
        # export:VAR=VALUE for the steps after it (e.g. export:GPU_MAX_HW_QUEUES=8, export:BSW_HP_INLINE_ENQ=1)
        export "${arg?}"; echo "exported $arg" ;;
    unset)
        unset "${arg?}"; echo "unset $arg" ;;
    py)
        # py:<file>[,arg,...] (commas for spaces)
        pa=($(sp "$arg"))
        log=$O/$(basename "${pa[0]}" .py)_$n.log
        timeout -k 10 600 python -u "${pa[@]}" > "$log" 2>&1 || fail "$step" $? "$log"
        tail -5 "$log" ;;
    *) echo "unknown step $step"; exit 2 ;;
    esac
    echo "== $step done in $(( $(date +%s) - t0 )) s"
done
