# build scattennet_amd/libscatten_hip_prev.so from a git revision's gemm.hip (default HEAD) and
# the current other objects — for tools/ab_lib.sh (same ABI required)
set -e
rev=${1:-HEAD}
d=$(mktemp -d)
mkdir -p $d/a/b $d/include
git show $rev:scattennet_amd/csrc/gemm.hip > $d/a/b/gemm.hip
git show $rev:scattennet_amd/csrc/common.h > $d/a/b/common.h
git show $rev:include/scatten.h > $d/include/scatten.h
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -c $d/a/b/gemm.hip -o $d/gemm.o
cd scattennet_amd/csrc
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $d/gemm.o build/attention.o build/rowops.o build/heads.o build/capi.o -o ../libscatten_hip_prev.so
rm -rf $d
