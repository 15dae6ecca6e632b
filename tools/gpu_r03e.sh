#!/bin/bash
# r03 (second session): the -m gpu suite, the driver-form bench, then the profile
# set (kernel trace + PMC passes) of the same tree, for profiles/r03.
set -e
TAG=${TAG:-r03e} bash tools/gpu_round.sh
bash tools/profile.sh r03
