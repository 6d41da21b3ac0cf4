#!/bin/bash
# GPU-box: a few reference configs through the CLI (1 round each), timing from metrics.jsonl.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in ${CONFIGS:-"fed_avg/cifar10.yaml fed_avg"}; do :; done
run() {
  local cfg=$1 grp=$2; shift 2
  local name=$(echo $cfg | tr '/' '_')
  timeout -k 10 ${CFG_TIMEOUT:-400} python simulator.py --config-name $cfg ++$grp.round=2 ++$grp.save_dir=gpurun_out/cfg_$name \
     ++$grp.log_level=WARNING "$@" > gpurun_out/cfg_$name.log 2>&1
  local rc=$?
  echo "rc=$rc" >> gpurun_out/cfg_$name.log
  return $rc
}
run fed_avg/cifar10.yaml fed_avg || exit $?
run fed_avg/mnist.yaml fed_avg || exit $?
run fed_avg/imdb.yaml fed_avg || exit $?
exit 0
