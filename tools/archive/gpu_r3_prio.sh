# stream-priority A/B at config 2: (plan knob cad_stream_prio, CadTrainer prio_stream) in {0,1}^2, alternated
set -o pipefail
mkdir -p gpurun_out
python -c "import torch; print('priority range', torch.cuda.Stream(priority=-1).priority, torch.cuda.Stream(priority=0).priority)" > gpurun_out/r03pr_range.log 2>&1
for rep in 1 2 3; do
  for v in 00 10 01 11; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --h2d-steps 0 --steps 30 --tune cad_stream_prio=${v:0:1} --prio-stream ${v:1:1} > gpurun_out/r03pr_${v}_$rep.log 2>&1 || exit 1
  done
done
