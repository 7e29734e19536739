#!/bin/bash
# r05ab: wave times of lone frames under the row orders and the measured tile order (probe build).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
O=gpurun_out/r05ab
mkdir -p $O
for v in "C3|2" "C3|3" "C4|0" "C4|3"; do
  c=${v%%|*}; o=${v#*|}
  RT_DISPATCH_ORDER=$o timeout -k 10 120 python tools/wave_times.py --lib uu-infogr-raytracer_amd/lib/ab/libraytracer_hip_wt.so \
      --config $c --batch 1 --reps 3 > $O/wt_${c}_order$o.txt 2>&1 || { tail $O/wt_${c}_order$o.txt; exit 1; }
  echo "== $c order $o"; grep "medians\|wave-us\|clock" $O/wt_${c}_order$o.txt
done
