set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/atomic_probe 1600 750 80 10 > gpurun_out/r03_atomic_probe.txt 2>&1 || exit 1
timeout -k 10 120 ./tools/atomic_probe 512 248 47 10 >> gpurun_out/r03_atomic_probe.txt 2>&1 || exit 1
