#!/bin/bash
# Dev: build the library of a git revision (default HEAD) into fccf-pcr_amd/lib_base/
# for interleaved A/B runs against the working tree's build (tools/ab_lib.sh base).
REV=${1:-HEAD}
WT=/tmp/fccf_base_wt
rm -rf $WT && git worktree prune && git worktree add -f --detach $WT $REV > /dev/null
make -C $WT/fccf-pcr_amd -j8 ARCH=gfx950 lib/libfccf.so > /tmp/fccf_base_build.log 2>&1 || { tail -20 /tmp/fccf_base_build.log; exit 1; }
mkdir -p fccf-pcr_amd/lib_base && cp $WT/fccf-pcr_amd/lib/libfccf.so fccf-pcr_amd/lib_base/libfccf.so
git worktree remove --force $WT
echo "lib_base = $(git rev-parse --short $REV)"
