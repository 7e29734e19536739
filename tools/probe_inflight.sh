set -o pipefail
cd $GRAFT_REPO_ROOT
for cfg in C2 C3; do
 for m in "16 2" "16 1" "32 1" "64 1" "128 1" "32 2"; do
  set -- $m
  timeout -k 10 120 python3 tools/frame_wall.py --config $cfg --batch $1 --inflight $2 --frames 1024 --reps 5 || exit 1
 done
done
