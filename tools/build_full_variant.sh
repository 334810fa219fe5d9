#!/bin/bash
# Build a whole-library experimental variant (every source recompiled with extra
# flags) into soundgen_beta_amd/lib/exp_<name>.so; select it at run time with
# SG_HIP_LIB=.../exp_<name>.so.   tools/build_full_variant.sh <name> <flags...>
set -e
cd "$(dirname "$0")/../soundgen_beta_amd/csrc"
name=$1; shift
mkdir -p _obj/v_$name
C="-O3 -std=c++17 -fPIC -Wall -Wno-unused-function -I../../include -I."
for f in *.cpp; do /opt/rocm/bin/hipcc $C "$@" -x c++ -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -c $f -o _obj/v_$name/${f%.cpp}.o & done
for f in *.hip; do /opt/rocm/bin/hipcc $C "$@" --offload-arch=gfx950 -ffp-contract=fast -fno-slp-vectorize -c $f -o _obj/v_$name/${f%.hip}.o & done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../lib/exp_$name.so _obj/v_$name/*.o
echo ../lib/exp_$name.so
