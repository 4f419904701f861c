#!/bin/bash
# kernel stats of config E (rasterizer time per 9 x 1080p views)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/pe -o run --output-format csv -- python3 bench.py --config E --steps 3 --warmup 1 --profile-only > $O/pe.log 2>&1 || { tail -20 $O/pe.log; exit 1; }
python3 - $O/pe/run_kernel_stats.csv <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:40]:
    n = r['Name']
    if any(k in n for k in ('rasterize', 'isect', 'radix', 'render_prep', 'pack_raster', 'tile_bins')):
        print(n[:60], r['Calls'], round(float(r['TotalDurationNs'])/1e6, 3), 'ms', round(float(r['AverageNs'])/1e3, 1), 'us')
PY
