# Builds lib/libdspcore_<NAME>.so with another per-phase instantiation list
# (A/B timing of k_chain_pp geometries with tools/gpu_libs.sh or ratio timing):
#   bash tools/build_pp_variant.sh NAME LIST_FILE
set -e
name=$1; list=$(realpath "$2")
cd "$(dirname "$0")/../dsp-audio-project_amd/csrc"
mkdir -p ../build/var
flags="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include -I. -fno-slp-vectorize -DPP_LIST=\"$list\""
objs=""
for f in abi src_poly iir fft fft_nf lfilter_nf audio_io; do objs="$objs ../build/$f.o"; done
for f in chain_tile chain_pp_0 chain_pp_1 chain_pp_2 chain_pp_3; do
  /opt/rocm/bin/hipcc $flags -c $f.hip -o ../build/var/${f}_$name.o &
  objs="$objs ../build/var/${f}_$name.o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../lib/libdspcore_$name.so $objs
echo built $name
