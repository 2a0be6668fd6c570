set -o pipefail
for cfg in "2 2 2" "2 4 4" "2 6 6" "4 4 4" "2 4 2" "2 2 4"; do
  set -- $cfg
  BLS_ML_G=$1 BLS_SIG_G=$2 BLS_H2C_G=$3 timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/gs.json 2>gpurun_out/gs.err || { tail -5 gpurun_out/gs.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/gs.json'));k=d['kernels_avg_ms'];print('ml=$1 sig=$2 h2c=$3', d['value'], 'sig_vm', k['sig_vm'], 'hash', k['fav_hash'], 'miller', k['miller'], 'msm', k['msm'])"
done
