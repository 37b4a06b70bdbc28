#!/bin/bash
# Two whole-step A/Bs and the tests that cover them: tools/r5_ab2.sh TAG
set -o pipefail
O=gpurun_out/${1:-r5w}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -k "overlap_optimizer or full4b_train_step_b32 or lm_head or ce" -x -v --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; tail -3 $O/pytest.txt; [ $rc -gt 1 ] && exit $rc
timeout -k 10 900 tools/ab_env.sh SVLA_OPT_OVERLAP 2 > $O/ab_opt.txt 2>&1 || exit $?
cat $O/ab_opt.txt
timeout -k 10 900 tools/ab_env.sh SVLA_LMHEAD_PIPE 2 1 4 > $O/ab_lmhead.txt 2>&1 || exit $?
cat $O/ab_lmhead.txt
