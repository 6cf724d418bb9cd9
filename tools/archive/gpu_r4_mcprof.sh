# kernel traces of the 3-D training configs (config 1 minicausal epoch, cad1 autoencoder step)
set -o pipefail
mkdir -p gpurun_out
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/mcp_cfg1 -o run -- python3 $ROOT/bench.py --config 1 --no-cpu-baseline --steps 10 > $ROOT/gpurun_out/mcp_cfg1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/mcp_cad1 -o run -- python3 $ROOT/bench.py --config cad1 --no-cpu-baseline --steps 10 > $ROOT/gpurun_out/mcp_cad1.log 2>&1
