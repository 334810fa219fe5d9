#!/bin/bash
# Build an experimental libsoundgen_hip variant: sg_harm.hip recompiled with extra
# flags, linked with the normal objects into soundgen_beta_amd/lib/exp_<name>.so
# (select at run time with SG_HIP_LIB=...).   tools/build_variant.sh <name> <flags...>
set -e
cd "$(dirname "$0")/../soundgen_beta_amd/csrc"
make -s
name=$1; shift
H="-O3 -std=c++17 -fPIC -Wall -Wno-unused-function -I../../include -I. --offload-arch=gfx950 -ffp-contract=fast -fno-slp-vectorize"
/opt/rocm/bin/hipcc $H "$@" -c ${SRC:-sg_harm.hip} -o _obj/sg_harm_$name.o
objs=$(ls _obj/*.o | grep -v 'sg_harm' ) 
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../lib/exp_$name.so $objs _obj/sg_harm_$name.o
echo ../lib/exp_$name.so
