#!/usr/bin/env bash
# TEST INFRASTRUCTURE ONLY.  Builds the reference simulator from its own source
# files where they lie under /root/reference/cpp (nothing is copied into this
# repo) plus our harness (oracle/ref_harness.cpp) into $MEV_REF_BUILD/libref_harness.so
# (default /tmp/marl_ref_build): OUTSIDE the repository tree, so nothing built from the
# reference can travel to the GPU box with a repository snapshot.
#
# Recipe notes:
#  * Only the simulation translation units are compiled: Car, Lidar, LineMask,
#    RoadMask, RouteGen, IntersectionEnv, TrafficFlow.  The renderer TUs
#    (Renderer.cpp, IntersectionEnv_render.cpp) and bindings.cpp are NOT built.
#  * IntersectionEnv.h includes Renderer.h, whose only content besides the class
#    declaration is a platform guard (`#ifndef _WIN32 #error`); -D_WIN32 passes
#    that guard.  No reference header is replaced or stubbed.
#  * The reference relies on MSVC's transitive size_t/uintptr_t; we force the
#    standard headers <cstddef>/<cstdint> with -include.
#  * ~IntersectionEnv() references Renderer::~Renderer() through a
#    unique_ptr<Renderer> that is null unless render() runs; we never render, so
#    that reference (in IntersectionEnv.o and in any TU that constructs an
#    IntersectionEnv) is made weak (objcopy --weaken-symbol) and resolves to
#    nothing.  No definition is supplied for it.
#  * -ffp-contract=off and no -march: the plain x86-64 SSE build, so golden
#    vectors are free of FMA contraction (SURVEY.md §7.3 hard part 2).
set -euo pipefail
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
REF="${MARL_REFERENCE_DIR:-/root/reference}/cpp"
OUT="${MEV_REF_BUILD:-/tmp/marl_ref_build}"
if [[ ! -f "$REF/IntersectionEnv.cpp" ]]; then
    echo "build_ref.sh: reference sources not found at $REF; skipping" >&2
    exit 0
fi
mkdir -p "$OUT/obj"
CXX="${CXX:-g++}"
FLAGS=(-O2 -std=c++17 -fPIC -ffp-contract=off -D_WIN32 -include cstddef -include cstdint -I "$REF")
for tu in Car Lidar LineMask RoadMask RouteGen IntersectionEnv TrafficFlow; do
    "$CXX" "${FLAGS[@]}" -c "$REF/$tu.cpp" -o "$OUT/obj/$tu.o"
done
"$CXX" "${FLAGS[@]}" -c "$HERE/ref_harness.cpp" -o "$OUT/obj/ref_harness.o"
for o in "$OUT"/obj/*.o; do
    objcopy --weaken-symbol=_ZN8RendererD1Ev --weaken-symbol=_ZN8RendererD2Ev "$o"
done
"$CXX" -shared -pthread -o "$OUT/libref_harness.so" "$OUT"/obj/*.o
echo "built $OUT/libref_harness.so"
