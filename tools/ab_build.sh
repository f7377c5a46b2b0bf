#!/bin/bash
# Build an A/B variant of the package into sound-event-detection_amd/build/ab/<name>
# (python sources copied, libsedx.so compiled with extra flags), for
# python bench.py --ab-package <that dir> ... in the same GPU call as the tree's build.
#   tools/ab_build.sh <name> "<extra hipcc flags>"
# (AB_ROOT=build/abx: a root .gpurunignore does not exclude, so the variant
# travels to the GPU box; build/ab stays local)
set -e
cd "$(dirname "$0")/.."
N=$1; X=$2
R=${AB_ROOT:-build/ab}
D=sound-event-detection_amd/$R/$N
mkdir -p $D/sedx $D/obj
cp sound-event-detection_amd/sedx/*.py $D/sedx/
make -s -C sound-event-detection_amd -j8 OBJDIR=$R/$N/obj EXTRA="$X" $R/$N/sedx/libsedx.so
ls -la $D/sedx/libsedx.so
