#!/bin/bash
# Repeated same-process A/Bs of several library builds with the order reversed
# every other repetition (pipelined, one-shot pair, one-shot single-lane), to
# separate <=1% effects from the run-to-run spread.
#   AB_LIBS="A.so B.so [C.so ...]"  AB_REPS (default 3)  AB_MODES (default "pipe pair single")
set -e
read -r -a LIBS <<< "$AB_LIBS"
REV=(); for ((i=${#LIBS[@]}-1; i>=0; i--)); do REV+=("${LIBS[$i]}"); done
for r in $(seq 1 ${AB_REPS:-3}); do
  if [ $((r % 2)) -eq 1 ]; then L="${LIBS[*]}"; else L="${REV[*]}"; fi
  for m in ${AB_MODES:-pipe pair single}; do
    echo "== rep $r $m"
    case $m in
      pipe)   AB_MODE=pipe timeout -k 10 200 python3 tools/ab_libs.py $L 2>&1 | grep -v amdgpu.ids ;;
      pair)   timeout -k 10 200 python3 tools/ab_libs.py $L 2>&1 | grep -v amdgpu.ids ;;
      single) FD_ED25519_GPU_PAIR=0 timeout -k 10 200 python3 tools/ab_libs.py $L 2>&1 | grep -v amdgpu.ids ;;
    esac
  done
done
