#!/bin/bash
# Prepare a built copy of the tree for an A/B or a diagnostic run (CPU side, before gpurun):
#   tools/mk_variant.sh prev [rev]   _ab/prev = git archive of <rev> (default HEAD), built
#   tools/mk_variant.sh tl           _ab/tl   = the working tree built with -DSBMP_TIMELINE
#                                              (k_step phase stamps, tools/timeline.py)
#   tools/mk_variant.sh <name> FLAGS _ab/<name> = the working tree built with SBMP_HIPCC_FLAGS=FLAGS
# _ab/ is git-ignored and travels to the GPU box with the snapshot.
set -euo pipefail
cd "$(dirname "$0")/.."
name=$1; shift || true
dst=_ab/$name
rm -rf "$dst" && mkdir -p "$dst"
if [ "$name" = prev ]; then
    git archive "${1:-HEAD}" | tar -x -C "$dst"
    flags=""
else
    tar --exclude=./_ab --exclude=./.git --exclude=./gpurun_out --exclude='*/_obj' --exclude='*.so' -cf - . | tar -xf - -C "$dst"
    if [ "$name" = tl ]; then flags=-DSBMP_TIMELINE; else flags="$*"; fi
fi
(cd "$dst" && SBMP_HIPCC_FLAGS="$flags" python3 -m cudasbmp_amd.build --force > /dev/null \
    && python3 -c "from oracle import pyoracle; pyoracle.build()" > /dev/null)
echo "$dst built (flags: ${flags:-none})"
