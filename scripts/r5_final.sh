#!/bin/bash
# final round-5 pass: full GPU tests + bench + rocprof + PMC (gpu_round.sh), then the configs
set -o pipefail
TAG=r5final2 TT=1000 scripts/gpu_round.sh || exit $?
TAG=r5final2_configs scripts/gpu_configs.sh || exit $?
