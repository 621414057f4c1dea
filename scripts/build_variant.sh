#!/bin/bash
# build a libsvhip.so variant with extra compile definitions (timing experiments):
#   bash scripts/build_variant.sh NAME -DSV_WGTIME=1 ...   ->  supervillain_amd/variants/libsvhip_NAME.so
set -e
name=$1; shift
cd $(dirname $0)/../supervillain_amd/csrc
mkdir -p ../variants/$name
PRIO="-mllvm --amdgpu-set-wave-priority"
[ "${NOPRIO:-0}" = 1 ] && PRIO=""  # (A/B: without the prologue wave-priority pass)
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math $PRIO -I../../include -I. $*"
objs=""
for f in capi plan mt19937 villain villain_hot villain_block villain_local worldline worldline_fused worldline_local domain replicas worm; do
  /opt/rocm/bin/hipcc $F -c $f.hip -o ../variants/$name/$f.o &
  objs="$objs ../variants/$name/$f.o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../variants/libsvhip_$name.so $objs -L/opt/rocm/lib -lrccl
rm -rf ../variants/$name
