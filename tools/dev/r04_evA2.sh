#!/bin/bash
# final evidence, part A with the small-graph A/B in front: current library vs var/libmgn_old.so
# (bitwise comparison, Cfg A / Cfg C rows), then tools/dev/r04_evA.sh
TAG=${1:-r04d}
bash tools/dev/small_ab.sh ${TAG}_ab old || exit 1
bash tools/dev/r04_evA.sh $TAG
