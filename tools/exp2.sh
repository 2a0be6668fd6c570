set -o pipefail
mkdir -p gpurun_out/exp2
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "resident" > gpurun_out/exp2/pytest.log 2>&1 || { tail -30 gpurun_out/exp2/pytest.log; exit 1; }
tail -2 gpurun_out/exp2/pytest.log
for mode in "" "--no-pipeline"; do
  timeout -k 10 240 python -u bench.py --steps 6 --warmup 2 --no-cpu $mode > gpurun_out/exp2/b$mode.json 2>gpurun_out/exp2/b$mode.err || { tail gpurun_out/exp2/b$mode.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/exp2/b$mode.json'));print('$mode',d['value'],d['ms_per_step'])"
done
GPU_MAX_HW_QUEUES=8 timeout -k 10 240 python -u bench.py --steps 6 --warmup 2 --no-cpu > gpurun_out/exp2/q8.json 2>gpurun_out/exp2/q8.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/exp2/q8.json'));print('q8',d['value'],d['ms_per_step'])"
GPU_MAX_HW_QUEUES=8 timeout -k 10 240 python -u bench.py --steps 6 --warmup 2 --no-cpu --no-profile > gpurun_out/exp2/q8np.json 2>gpurun_out/exp2/q8np.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/exp2/q8np.json'));print('q8 noprof',d['value'],d['ms_per_step'])"
