# build scattennet_amd/libscatten_hip_prev.so from a git revision's copy of one kernel source
# (SRC, default gemm) and the current other objects — for tools/ab_lib.sh (same ABI required)
set -e
rev=${1:-HEAD}
src=${SRC:-gemm}
d=$(mktemp -d)
mkdir -p $d/a/b $d/include
git show $rev:scattennet_amd/csrc/$src.hip > $d/a/b/$src.hip
git show $rev:scattennet_amd/csrc/common.h > $d/a/b/common.h
git show $rev:include/scatten.h > $d/include/scatten.h
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -c $d/a/b/$src.hip -o $d/$src.o
cd scattennet_amd/csrc
objs="$d/$src.o"
for o in gemm attention rowops heads; do [ $o = $src ] || objs="$objs build/$o.o"; done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs build/capi.o -o ../libscatten_hip_prev.so
rm -rf $d
