cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/ab.sh 3 || exit 1
bash scripts/ab.sh 1 --worlds 4096 --steps 200 || exit 1
bash scripts/pmc_vars.sh "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS"
