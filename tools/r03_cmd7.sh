set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_fortran.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03_fortran.log 2>&1 || exit 1
bash tools/r03_cmd6.sh
