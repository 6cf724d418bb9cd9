# print medians of A/B tags from gpurun_out (tools/ab_knob.sh / ab_so.sh logs)
for t in "$@"; do
  python tools/ab_summary.py $t 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print('$t', d['A']['median_ms'], d['B']['median_ms'], [r['ms_per_step'] for r in d['A']['runs']], [r['ms_per_step'] for r in d['B']['runs']])" 2>/dev/null || echo "$t: no data"
done
