# alternative builds of libllp_hip.so for ablations (tools/bin/<name>/libllp_hip.so): NOSTORE, NOEPI
set -e
cd "$(dirname "$0")/.."
for v in NOSTORE NOEPI; do
  d=tools/bin/$v; mkdir -p $d/obj
  for f in linkless-link-prediction_amd/csrc/*.hip linkless-link-prediction_amd/csrc/*.cpp; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I include -I linkless-link-prediction_amd/csrc \
      -Wno-unused-result -munsafe-fp-atomics -DLLP_ABLATE_$v -c $f -o $d/obj/$(basename $f).o &
  done
  wait
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $d/obj/*.o -o $d/libllp_hip.so
done
