# G (items per VM workgroup) sweep on the pipelined bench
set -o pipefail
mkdir -p gpurun_out/gs2
run() {
  env "$@" timeout -k 10 120 python -u bench.py --steps 8 --warmup 3 --no-cpu --no-profile > gpurun_out/gs2/o.json 2>gpurun_out/gs2/e.log || { tail -5 gpurun_out/gs2/e.log; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/gs2/o.json'));print('$*',d['value'],d['ms_per_step'])"
}
run X=1
run BLS_H2C_G=4
run BLS_H2C_G=6
run BLS_SIG_G=6
run BLS_SIG_G=2
run BLS_M2_G=1
run BLS_ML_G=1
