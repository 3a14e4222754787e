#!/bin/bash
# GRM loci-split sweep at C2 (GBM_GRM_SPLIT overrides the planner): time_grm.py per candidate.
set -o pipefail
export PYTHONUNBUFFERED=1
SPLITS=${SPLITS:-"auto 2343,548,164,49,21 2700,300,90,35 2000,700,300,100,25 1,1 2500,400,150,50,25 1 2200,600,200,80,30,15 1,1,1"}
for S in $SPLITS; do
  if [ "$S" = auto ]; then unset GBM_GRM_SPLIT; else export GBM_GRM_SPLIT=$S; fi
  echo -n "split $S: "; timeout -k 10 120 python tools/time_grm.py ${NP:-5000 50000} || exit 1
done
