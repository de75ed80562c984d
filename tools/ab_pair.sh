# interleaved A/B of libzgpu builds on the bench's 4096 x 1 MiB L6 sub-batch (tools/ab_match.py), two passes:
#   bash tools/ab_pair.sh reps libA.so libB.so [libC.so ...]
set -e
R=$1; shift
for k in 1 2; do
  for L in "$@"; do timeout -k 10 240 python3 -u tools/ab_match.py $L $R; done
done
