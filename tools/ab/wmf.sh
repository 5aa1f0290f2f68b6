# WMF A/B: 1080p launch time and output checksum of each build, twice
# usage: bash tools/ab/wmf.sh LIB...
set -e
: > gpurun_out/wmf_ab.log
for i in 1 2; do
for L in "$@"; do
  echo "== $L" >> gpurun_out/wmf_ab.log
  timeout -k 10 120 python -u tools/wmf_bench.py --lib $L >> gpurun_out/wmf_ab.log 2>&1
done; done
