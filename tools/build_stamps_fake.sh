#!/bin/bash
# Diagnostic timing build: the single-lane decoders with clock stamps AND no global loads
# (-DTDECS_FAKELOAD: results are garbage) -> srsran_4g_amd/lib/stamps_fake/libsrsran_4g_amd.so.
# Compared with lib/stamps/ by tools/tdec_stamps.py --lib, it isolates the cycles the window loads cost.
set -e
cd "$(dirname "$0")/../srsran_4g_amd/csrc"
make -j8 >/dev/null
D=../lib/stamps_fake
mkdir -p $D
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -Wno-unused-value -DTDECS_STAMPS -DTDECS_FAKELOAD"
/opt/rocm/bin/hipcc $F -DTDECS_NSB=16 -c tdecs_kernel.hip -o $D/tdec16s_kernel.o &
/opt/rocm/bin/hipcc $F -DTDECS_NSB=8 -c tdecs_kernel.hip -o $D/tdec8s_kernel.o &
/opt/rocm/bin/hipcc $F -DTDECS_NSB=16 -DTDECS_W=8 -c tdecs_kernel.hip -o $D/tdec16sw8_kernel.o &
/opt/rocm/bin/hipcc $F -DTDECS_NSB=8 -DTDECS_W=8 -c tdecs_kernel.hip -o $D/tdec8sw8_kernel.o &
/opt/rocm/bin/hipcc $F -c tdec_api.cpp -o $D/tdec_api.o &
wait
REST=$(ls ../lib/*.o | grep -v -E "/(tdec16s|tdec8s|tdec16sw8|tdec8sw8)_kernel.o|/tdec_api.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,--version-script=exports.map -o $D/libsrsran_4g_amd.so $D/*.o $REST
echo built $D/libsrsran_4g_amd.so
