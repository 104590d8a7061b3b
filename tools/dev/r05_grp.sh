#!/bin/bash
# Round 5 (reverted experiment: the MGN_CONC_GROUP knob it sets was removed after this A/B, profiles/r05_ab.txt): one side-stream hand-over per group of blocks, bf16 Cfg B, one box.
bash tools/dev/r05_env.sh grp "MGN_CONC_GROUP=2" "MGN_CONC_GROUP=3" "MGN_CONC_GROUP=5"
