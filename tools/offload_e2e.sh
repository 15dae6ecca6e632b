#!/bin/bash
# Two-process run of the GPU offload link (run via gpurun from the repo root):
# the server (owns the GPU) in the background, the client (no GPU) in front.
set -e
mkdir -p gpurun_out
NAME=/fdvo_e2e_$$
timeout -k 10 300 ./firedancer_amd/fd_verify_offload_server --name $NAME --batch ${BATCH:-65536} --threads ${THREADS:-16} \
  > gpurun_out/offload_server.json 2> gpurun_out/offload_server.err &
SRV=$!
# the client's clock starts at its first publish: wait for the server's readiness line
for i in $(seq 600); do grep -q ready gpurun_out/offload_server.json 2>/dev/null && break; kill -0 $SRV 2>/dev/null || break; sleep 0.2; done
timeout -k 10 240 python3 tools/bench_offload.py --name $NAME ${CLIENT_ARGS} > gpurun_out/offload_client.json 2> gpurun_out/offload_client.err || { kill $SRV; wait $SRV; exit 1; }
wait $SRV
cat gpurun_out/offload_client.json gpurun_out/offload_server.json
