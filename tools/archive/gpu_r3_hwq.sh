set -o pipefail
for rep in 1 2; do
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/r03hw_A_$rep.log 2>&1 || exit 1
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/r03hw_B_$rep.log 2>&1 || exit 1
done
