#!/bin/bash
# Build an A/B variant of the package into sound-event-detection_amd/build/ab/<name>
# (python sources copied, libsedx.so compiled with extra flags), for
# python bench.py --ab-package <that dir> ... in the same GPU call as the tree's build.
#   tools/ab_build.sh <name> "<extra hipcc flags>"
set -e
cd "$(dirname "$0")/.."
N=$1; X=$2
D=sound-event-detection_amd/build/ab/$N
mkdir -p $D/sedx $D/obj
cp sound-event-detection_amd/sedx/*.py $D/sedx/
make -s -C sound-event-detection_amd -j8 OBJDIR=build/ab/$N/obj EXTRA="$X" build/ab/$N/sedx/libsedx.so
ls -la $D/sedx/libsedx.so
