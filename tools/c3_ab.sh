set -e
mkdir -p gpurun_out/c3ab
for rep in 1 2; do
for L in tools/bin/lib_base.so tools/bin/lib_F.so; do
  b=$(basename $L .so)
  FD_ED25519_GPU_LIB=$L timeout -k 10 200 python3 bench.py --config 3 --steps 10 --warmup 3 --no-cpu > gpurun_out/c3ab/${b}_pipe_$rep.json 2>/dev/null
  FD_ED25519_GPU_LIB=$L timeout -k 10 200 python3 bench.py --config 3 --pipeline 0 --steps 10 --warmup 3 --no-cpu > gpurun_out/c3ab/${b}_launch_$rep.json 2>/dev/null
  python3 -c "
import json,sys
for m in ('pipe','launch'):
    d=json.loads(open('gpurun_out/c3ab/${b}_'+m+'_$rep.json').read().strip().splitlines()[-1]); print('$b', m, $rep, round(d['value']/1e6,2))"
done; done
