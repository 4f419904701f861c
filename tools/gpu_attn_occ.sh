#!/bin/bash
# attention occupancy variants: kernel stats of the config-B bench with the default library and exp_occ5.so
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out
for v in base occ5; do
  if [ $v = base ]; then L=splatformer_amd/libsfx.so; else L=splatformer_amd/exp_$v.so; fi
  SFX_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ao_$v -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --profile-only > $O/ao_$v.log 2>&1 || { tail -20 $O/ao_$v.log; exit 1; }
  python3 - "$O/ao_$v/run_kernel_stats.csv" $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'window_attn' in r['Name']: print(sys.argv[2], r['Name'][:60], r['Calls'], round(float(r['TotalDurationNs'])/1e6, 3), 'ms', round(float(r['AverageNs'])/1e3, 1), 'us')
PY
done
