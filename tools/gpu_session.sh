set -e
mkdir -p gpurun_out/ls
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for V in 1 0; do
  FD_ED25519_GPU_LENSORT=$V timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAVES SQ_INSTS_VMEM_RD --output-format csv -d gpurun_out/ls/v$V -o pmc -- python3 bench.py --config 3 --steps 3 --warmup 1 --no-cpu --pipeline 0 > /dev/null 2> gpurun_out/ls/v$V.err
  python3 tools/pmc_summary.py gpurun_out/ls/v$V/pmc_counter_collection.csv mid
done
