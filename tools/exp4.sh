set -o pipefail
mkdir -p gpurun_out/exp4
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/exp4/pytest.log 2>&1 || { tail -30 gpurun_out/exp4/pytest.log; exit 1; }
tail -2 gpurun_out/exp4/pytest.log
run() {
  env "$@" timeout -k 10 120 python -u bench.py --steps 8 --warmup 3 --no-cpu --no-profile > gpurun_out/exp4/o.json 2>gpurun_out/exp4/e.log || { tail -5 gpurun_out/exp4/e.log; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/exp4/o.json'));print('$*',d['value'],d['ms_per_step'])"
}
run X=1
run BLS_H2C_G=4 BLS_XC_G=6
run BLS_XC_G=6
run BLS_H2C_G=4
run BLS_SIG_G=6
