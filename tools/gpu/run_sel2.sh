cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/x; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_lagged.py tests/test_gpu_parity.py -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/x/pytest.log 2>&1 || { tail -20 gpurun_out/x/pytest.log; exit 1; }
tail -1 gpurun_out/x/pytest.log
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/x/pmc_fetch -o pmc -- python tools/pmc_run.py > gpurun_out/x/pmc_fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/x/pmc_write -o pmc -- python tools/pmc_run.py > gpurun_out/x/pmc_write.log 2>&1 || exit 1
python tools/pmc_summarize.py gpurun_out/x/pmc_fetch/pmc_counter_collection.csv gpurun_out/x/pmc_write/pmc_counter_collection.csv > gpurun_out/x/pmc.json
python -c "import json; d=json.load(open('gpurun_out/x/pmc.json')); print({k: round(v['hbm_bytes_per_launch']) for k,v in d.items() if k!='_note'})"
timeout -k 10 300 python bench.py --cpu-minibatches 0 > gpurun_out/x/bench.json 2> gpurun_out/x/bench.err || exit 1
python -c "
import json
for l in open('gpurun_out/x/bench.json'):
    if l.startswith('{'): d=json.loads(l); print(d['value'], d['stages_us'], d['phases_ms'])"
