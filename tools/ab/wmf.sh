# WMF A/B: 1080p launch time and output checksum, baseline vs variant, twice
set -e
: > gpurun_out/wmf_ab.log
for i in 1 2; do
for L in optical-flow-python_amd/optical_flow/_lib/liboptflow.so "$@"; do
  echo "== $L" >> gpurun_out/wmf_ab.log
  timeout -k 10 120 python -u tools/wmf_bench.py --lib $L >> gpurun_out/wmf_ab.log 2>&1
done; done
