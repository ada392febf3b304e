# Build A/B variants of the fused MAPPO gradient kernel: mg_variants.sh name "flags" [name "flags" ...]
# -> mini-marl_amd/lib/var_<name>.so (load with MM_LIB=...)
set -e
cd "$(dirname "$0")/../mini-marl_amd"
make -s -j8 lib/libminimarl.so
mkdir -p build/var
OTHERS=$(ls build/*.o | grep -v mappo_grad.o | grep -v torch_ops.o)
while [ $# -gt 1 ]; do
  n=$1; f=$2; shift 2
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../include -Icsrc $f -c csrc/mappo_grad.hip -o build/var/mg_$n.o &
done
wait
for o in build/var/mg_*.o; do n=$(basename $o .o); n=${n#mg_}; /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o lib/var_$n.so $OTHERS $o; done
ls lib/var_*.so
