#!/bin/bash
# Build an A/B variant of the engine library into _ab/<name>/ (CPU side):
#   bash tools/build_variant.sh <name> "<hipcc flags for psx_sweep3 only>" ["<hipcc flags for every object>"] [source dir]
set -e
name=$1; k3=$2; extra=$3; src=${4:-pipsort_amd}
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d /tmp/psxvar.XXXX)
mkdir -p "$T/pipsort_amd"
cp -r "$R/$src/csrc" "$R/$src/Makefile" "$T/pipsort_amd/"
cp -r "$R/include" "$T/"
make -s -j 8 -C "$T/pipsort_amd" lib/libpipsort_engine.so \
  HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -Wno-unused-value -Wno-unused-result $extra" K3FLAGS="$k3"
mkdir -p "$R/_ab/$name"
cp "$T/pipsort_amd/lib/libpipsort_engine.so" "$R/_ab/$name/"
rm -rf "$T"
echo "built _ab/$name (k3: $k3; all: $extra)"
