#!/bin/bash
# A/B of two library builds (LVX_LIB_PATH): bench configs[1] (and configs[2] with AB_C2=1),
# alternating, 3 rounds. usage: bash tools/ab_lib.sh BASE_SO NEW_SO
set -o pipefail
export PYTHONPATH=.
mkdir -p gpurun_out
for i in 1 2 3; do for so in "$1" "$2"; do for c in ${AB_CONFIGS:-1 ${AB_C2:+2}}; do
  ex=""; [ "$c" == "2" ] && ex="--steps 2"; [ "$c" == "4" ] && ex="--steps 8"
  LVX_LIB_PATH=$so timeout -k 10 200 python bench.py --config $c $ex --no-cpu-baseline > gpurun_out/ab.json 2>/dev/null || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]); print('c$c', '$so', d['value'], d['ms_per_step'], {k: v['avg_us'] for k, v in d['kernels'].items()})"
done; done; done
