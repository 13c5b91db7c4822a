#!/bin/bash
# Build libpquic_fec.so from the sources of another commit (A/B baselines):
#   bash tools/build_at_commit.sh COMMIT OUT.so
set -e
C=$1; OUT=$(realpath -m $2)
W=/tmp/pquic_wt_$C
rm -rf $W && mkdir -p $W
git archive $C pquic_amd include | tar -x -C $W
python3 -c "import sys; sys.path.insert(0, '$W'); from pquic_amd import build as b; b.build(out='$OUT')"
echo built $OUT from $C
