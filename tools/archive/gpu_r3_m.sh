# round 3 (m): cross-stream latency probe, dir_mid phase cycles, chain marks
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./tools/exp/xstream_probe > gpurun_out/r3m_xstream.txt 2>&1 && \
timeout -k 10 200 python -u tools/exp/chain_marks.py head_dbg=1 > gpurun_out/r3m_marks.txt 2>&1
