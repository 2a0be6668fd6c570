set -o pipefail
mkdir -p gpurun_out/exp3
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "resident" > gpurun_out/exp3/pytest.log 2>&1 || { tail -30 gpurun_out/exp3/pytest.log; exit 1; }
tail -2 gpurun_out/exp3/pytest.log
for q in 4 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 240 python -u bench.py --steps 8 --warmup 3 --no-cpu > gpurun_out/exp3/q$q.json 2>gpurun_out/exp3/q$q.err || { tail gpurun_out/exp3/q$q.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/exp3/q$q.json'));print('q$q',d['value'],d['ms_per_step'])"
done
