#!/bin/bash
# a round's closing GPU pass: full GPU tests + bench + rocprof + PMC (gpu_round.sh), then the
# other BASELINE configurations (gpu_configs.sh).   TAG=<name> scripts/final_pass.sh
set -o pipefail
TAG=${TAG:?TAG} TT=${TT:-1000} scripts/gpu_round.sh || exit $?
TAG=${TAG}_configs scripts/gpu_configs.sh || exit $?
