#!/bin/bash
# Build an experimental libsoundgen_hip variant: one kernel source (SRC, default
# sg_harm.hip; REPLACES names the object it stands in for) recompiled with extra
# flags, linked with the normal objects into soundgen_beta_amd/lib/exp_<name>.so
# (select at run time with SG_HIP_LIB=...).   tools/build_variant.sh <name> <flags...>
set -e
cd "$(dirname "$0")/../soundgen_beta_amd/csrc"
make -s
name=$1; shift
H="-O3 -std=c++17 -fPIC -Wall -Wno-unused-function -I../../include -I. --offload-arch=gfx950 -ffp-contract=fast -fno-slp-vectorize"
src=${SRC:-sg_harm.hip}
rep=${REPLACES:-$(basename $src .hip)}
mkdir -p _obj/var
/opt/rocm/bin/hipcc $H "$@" -c $src -o _obj/var/${rep}_$name.o
objs=$(ls _obj/*.o | grep -v "/$rep.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../lib/exp_$name.so $objs _obj/var/${rep}_$name.o
echo ../lib/exp_$name.so
