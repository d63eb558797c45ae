#!/bin/sh
# r06_final.sh TAG — round-end evidence on one box: the -m gpu suite, smoke(), the default bench line, its
# rocprofv3 --kernel-trace --stats, serial + concurrent traces of one C4 update, and every config's line
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
sh tools/round_check.sh $1 || exit 1
sh tools/trace_config.sh $1_trace "" || exit 1
cd $R && sh tools/final_configs.sh $1_cfg || exit 1
