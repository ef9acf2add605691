#!/bin/bash
# Dev: build the library of git revision $1 into fccf-pcr_amd/lib_$2/ (bisecting with
# FCCF_LIB=fccf-pcr_amd/lib_$2/libfccf.so python tools/quick_perf.py).
REV=$1
NAME=$2
WT=/tmp/fccf_rev_wt_$NAME
rm -rf $WT && git worktree prune && git worktree add -f --detach $WT $REV > /dev/null
make -C $WT/fccf-pcr_amd -j8 ARCH=gfx950 lib/libfccf.so > /tmp/fccf_rev_$NAME.log 2>&1 || { tail -20 /tmp/fccf_rev_$NAME.log; exit 1; }
mkdir -p fccf-pcr_amd/lib_$NAME && cp $WT/fccf-pcr_amd/lib/libfccf.so fccf-pcr_amd/lib_$NAME/libfccf.so
git worktree remove --force $WT
echo "lib_$NAME = $(git rev-parse --short $REV)"
