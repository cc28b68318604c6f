# round 5: what in the process state slows the next bench leg (tools/leg_probe.py sequences, one process each)
set -o pipefail
mkdir -p gpurun_out/r5y
cd $GRAFT_REPO_ROOT
export HISEG_BENCH_STEP_TIMES=1
i=0
for seq in copy,infer,mem,copy,distill,copy \
           copy,infer_serial,mem,copy,distill \
           infer,empty,copy,distill \
           copy,mem,train,mem,copy,empty,copy,sleep:5,copy,sleep:10,copy,sleep:20,copy,infer \
           train,copy,infer,distill,mem; do
  i=$((i+1))
  echo "## $seq" >> gpurun_out/r5y/probe.txt
  timeout -k 10 400 python3 -u tools/leg_probe.py $seq >> gpurun_out/r5y/probe.txt 2> gpurun_out/r5y/err$i.txt || exit $?
done
