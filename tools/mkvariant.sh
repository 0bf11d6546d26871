#!/bin/bash
# Build an A/B variant of the working tree into _ab/<name> with extra -D defines:
#   tools/mkvariant.sh <name> [MACRO[=value] ...]
set -e
name=$1; shift
rm -rf _ab/$name && mkdir -p _ab/$name
tar --exclude=./_ab --exclude=./.git --exclude=./gpurun_out --exclude='*/_obj' -cf - . | tar -xf - -C _ab/$name
defs=""
for m in "$@"; do defs="$defs#define $m\n"; done
f=_ab/$name/cudasbmp_amd/csrc/kgmt_kernels.hip
printf "$defs" | sed 's/=/ /' | cat - $f > $f.new && mv $f.new $f
(cd _ab/$name && python3 -m cudasbmp_amd.build --force > /dev/null) || { echo "build failed"; exit 1; }
echo "built _ab/$name with: $*"
