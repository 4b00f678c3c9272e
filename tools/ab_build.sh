#!/bin/bash
# Build libdqdk_gpu.so from a git revision (or the working tree: "wt") into
# build/ab/<name>.so for same-box A/B timing (tools/ab_run.sh).
# usage: bash tools/ab_build.sh <name> <rev|wt> [<file>=<rev> ...]  (per-file overrides, e.g.
#        dqdk_amd/csrc/rx_kernels.hip=HEAD: the working tree with that file as committed)
set -e
name=$1; rev=$2; shift 2
root=$(cd "$(dirname "$0")/.." && pwd)
src=/tmp/dqdk_ab_$name
rm -rf $src && mkdir -p $src/dqdk_amd/csrc $src/include $root/build/ab
if [ "$rev" = wt ]; then
    cp $root/dqdk_amd/csrc/* $src/dqdk_amd/csrc/ && cp $root/include/* $src/include/
else
    git -C $root archive $rev dqdk_amd/csrc include | tar -x -C $src
fi
for ov in "$@"; do
    git -C $root show "${ov#*=}:${ov%%=*}" > $src/${ov%%=*}
done
objs=""
for f in $src/dqdk_amd/csrc/*.hip; do
    o=$src/$(basename $f .hip).o
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -DDQDK_AB_VARIANTS $EXTRA_FLAGS -c $f -o $o
    objs="$objs $o"
done
for f in $src/dqdk_amd/csrc/*.c; do
    o=$src/$(basename $f .c)_c.o
    gcc -O3 -fPIC -std=gnu11 -pthread -c $f -o $o
    objs="$objs $o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $root/build/ab/$name.so $objs -lpthread
echo built build/ab/$name.so
