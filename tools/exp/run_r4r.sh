set -o pipefail
mkdir -p gpurun_out/r4r && export TMPDIR=/tmp
timeout -k 10 1150 python -u tools/nmse_curves.py --dim 4194304 --instances 15 --users 1,6,11,51,101 --out gpurun_out/r4r/nmse_curves_d4194304_i15.json > gpurun_out/r4r/nmse.log 2>&1
