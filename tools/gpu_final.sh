#!/bin/bash
# Round-end validation in one GPU call: the whole -m gpu suite, smoke(),
# configs 2 and 3 in the driver's form back to back (same box), and the
# effective clock (GRBM_GUI_ACTIVE) of a long config-2 run (80 steps, ~44 ms)
# beside config 3's (3 steps of ~9 ms), so their clocks compare at similar
# run lengths.  Stops at the first failure.
set -e
mkdir -p gpurun_out/final
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/final
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 > $O/c2_$r.json 2> $O/c2_$r.err
  timeout -k 10 300 python3 bench.py --config 3 --steps 20 --warmup 5 > $O/c3_$r.json 2> $O/c3_$r.err
done
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/grbm_c2long -o pmc -- python3 bench.py --steps 80 --warmup 1 --no-cpu > /dev/null 2> $O/grbm_c2long.err
timeout -s KILL 180 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/grbm_c3 -o pmc -- python3 bench.py --config 3 --steps 3 --warmup 1 --no-cpu > /dev/null 2> $O/grbm_c3.err
echo done > $O/DONE
