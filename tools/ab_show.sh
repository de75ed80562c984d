# print the A/B results of tools/ab_match.sh
for f in gpurun_out/v*_tests.log; do echo "$f: $(tail -2 $f | head -1)"; done
grep -h "stats" gpurun_out/v*_stats.err 2>/dev/null
for f in gpurun_out/ab_v*.json; do python3 -c "
import json,sys; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['verified']['deflate_buffers_bit_exact_vs_oracle'])"; done
