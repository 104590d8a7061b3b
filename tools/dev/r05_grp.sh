#!/bin/bash
# Round 5: side-stream hand-over per group of blocks (MGN_CONC_GROUP), bf16 Cfg B, one box.
bash tools/dev/r05_env.sh grp "MGN_CONC_GROUP=2" "MGN_CONC_GROUP=3" "MGN_CONC_GROUP=5"
