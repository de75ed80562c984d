#!/bin/bash
# A/B of k_links: head[] in the key region, two workgroups per CU (ZGPU_LINKS_GH=1, default) against head[] in LDS
set -o pipefail
O=gpurun_out/${R:-r05m}
mkdir -p $O
export TMPDIR=/tmp
for k in 1 2; do
  for m in 1 0; do
    ZGPU_LINKS_GH=$m timeout -k 10 300 python3 -u bench.py --no-cpu --no-inflate --steps 3 --warmup 1 > $O/ab_$m.$k.json 2> $O/ab_$m.$k.err || { echo "bench failed"; tail -20 $O/ab_$m.$k.err; exit 1; }
    python3 -c "import json; d=[json.loads(l) for l in open('$O/ab_$m.$k.json') if l.startswith('{')][-1]; print('gh=$m', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['verified']['deflate_buffers_bit_exact'], d['stage_ms_per_step'])"
  done
done
for m in 1 0; do
  ZGPU_NO_PIPELINE=1 ZGPU_LINKS_GH=$m timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k$m -o run -- python3 bench.py --no-cpu --no-inflate --steps 2 --warmup 1 --buffers 8192 --crc-buffers 4096 --adler-buffers 0 > $O/k$m.json 2> $O/k$m.err || { echo "rocprof failed"; tail -5 $O/k$m.err; exit 1; }
  echo "gh=$m"; grep -E "k_links|k_count|k_match" $(find $O/k$m -name "*kernel_stats.csv")
done
