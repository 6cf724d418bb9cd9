# round-3 build (ab/r03: git archive of the round-3 verdict commit, built here) against this tree, back to back on one box
set -o pipefail
mkdir -p gpurun_out
R=$(pwd)
run() {  # cfg tree tag
  if [ $2 = r03 ]; then d=$R/ab/r03; else d=$R; fi
  (cd $d && timeout -k 10 200 python bench.py --config $1 --no-cpu-baseline > $R/gpurun_out/vs_$1_$2_$3.json 2>/dev/null)
}
run 2 r03 a && run 2 r04 a && run 2 r03 b && run 2 r04 b && \
run 4 r03 a && run 4 r04 a && run 1 r03 a && run 1 r04 a && run cad1 r03 a && run cad1 r04 a
