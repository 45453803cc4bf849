#!/bin/bash
# Host-buffer pipeline steady state: 10 calls per process (median of the last 7), the round-3
# pipeline (early start: chunk 0 before the rest of the prepass) vs BSW_HP_NO_EARLY; x3.
# (The first version of this A/B also folded the remainder chunk into the last one: slower,
# removed -- profiles/r03/hostpath_steady_ab.txt keeps both.)
set -o pipefail
O=gpurun_out/r3w; mkdir -p $O
for rep in 1 2 3; do
  line="rep $rep"
  for v in new old; do
    case $v in new) E="";; old) E="BSW_HP_NO_EARLY=1";; esac
    timeout -k 10 200 env $E python3 tools/host_path_once.py 262144 10 > $O/${v}_$rep.log 2>&1 || { tail $O/${v}_$rep.log; exit 1; }
    med=$(grep '^call' $O/${v}_$rep.log | tail -7 | awk '{print $2}' | sort -n | sed -n 4p)
    line="$line | $v median $med ms"
  done
  echo "$line"
done
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench.log').read().strip().splitlines()[-1]);print(d['value'], d['abi_inclusive_value'], d['abi_inclusive']['ms_all_calls'], [ (c['pairs_per_call'], c['M_pairs_per_s_8_callers']) for c in d['abi_inclusive']['per_call_curve_cpp_callers']['curve']])"
