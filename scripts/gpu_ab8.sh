#!/bin/bash
# A/B of unmask variants 0 (default) and 8 (aligned loads) on C4, C2, C5.
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out
mkdir -p $OUT
for c in ${AB_CONFIGS:-c4 c2 c5}; do
  timeout -k 10 300 python tools/ab_unmask.py --config $c --variants ${AB_VARIANTS:-0,8} --grids 0 --rounds 5 --reps 3 \
    > $OUT/ab8_$c.log 2> $OUT/ab8_$c.err || { tail -5 $OUT/ab8_$c.err; exit 1; }
  python - "$OUT/ab8_$c.log" "$c" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[2], [(v["variant"], v["unmask_ms_median"], v["GBps"]) for v in d["variants"]],
      d["stream_copy_ceiling"])
PY
done
