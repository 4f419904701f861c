cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/gemm_tune.py > gpurun_out/tune_sk.jsonl 2> gpurun_out/tune_sk.err || { tail -20 gpurun_out/tune_sk.err; exit 1; }
for i in 1 2; do timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/sk_bench$i.json 2>gpurun_out/sk_bench.err || exit 1; python3 -c "import json;d=json.load(open('gpurun_out/sk_bench$i.json'));print(d['value'],d['ms_per_step'],d['roofline']['gemm_ms_per_scene'])"; done
