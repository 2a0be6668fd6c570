set -o pipefail
mkdir -p gpurun_out/exp1
for b in 5000 10000 20000 40000; do
  timeout -k 10 240 python -u bench.py --steps 4 --warmup 1 --no-cpu --batch $b > gpurun_out/exp1/b$b.json 2>gpurun_out/exp1/b$b.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/exp1/b$b.json'));print($b,d['value'],d['ms_per_step'])"
done
GPU_MAX_HW_QUEUES=8 timeout -k 10 240 python -u bench.py --steps 4 --warmup 1 --no-cpu > gpurun_out/exp1/q8.json 2>gpurun_out/exp1/q8.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/exp1/q8.json'));print('q8',d['value'],d['ms_per_step'])"
