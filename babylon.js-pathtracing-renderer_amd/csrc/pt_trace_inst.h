// pt_trace_inst.h — explicit instantiations of pt_trace / pt_persist (pt_trace.h) for the program
// variants of one BVH walk, and their launchers; included by pt_trace_walk_<walk>.hip with
// PT_WALK_NAME / PT_WALK_PROGS set, so that the walks' variants compile as parallel translation units.
#include "pt_trace.h"

#define PT_CAT2(a, b) a##b
#define PT_CAT(a, b) PT_CAT2(a, b)

namespace pt {
// the megakernel variant of a draw: counting, timed, or timed with late-bounce compaction (mesh programs)
template <int P>
hipError_t launchTrace(int count, bool cont, const TraceArgs* a, dim3 grid, dim3 block, hipStream_t s)
{
    if (count) hipLaunchKernelGGL((pt_trace<P, true, false>), grid, block, 0, s, *a);
    else if constexpr (kHasMesh<P>) {
        if (cont) hipLaunchKernelGGL((pt_trace<P, false, true>), grid, block, 0, s, *a);
        else hipLaunchKernelGGL((pt_trace<P, false, false>), grid, block, 0, s, *a);
    } else hipLaunchKernelGGL((pt_trace<P, false, false>), grid, block, 0, s, *a);
    return hipGetLastError();
}
template <int P>
hipError_t launchCont(const TraceArgs* a, dim3 grid, hipStream_t s)
{
    if constexpr (kHasMesh<P>) {
        hipLaunchKernelGGL((pt_cont<P>), grid, dim3(kTraceBlock), 0, s, *a);
        return hipGetLastError();
    }
    return hipErrorInvalidValue;
}
#define PT_INST(P)                                                                                          \
    template __global__ void pt_persist<P, false>(TraceArgs, WfBufs, int, unsigned, unsigned, unsigned);    \
    template __global__ void pt_persist<P, true>(TraceArgs, WfBufs, int, unsigned, unsigned, unsigned);
PT_WALK_PROGS(PT_INST)
#undef PT_INST
} // namespace pt

hipError_t PT_CAT(pt_launch_trace_, PT_WALK_NAME)(int prog, int count, const pt::TraceArgs* a, dim3 grid, dim3 block,
                                                  hipStream_t s)
{
    using namespace pt;
    const bool cont = a->cont_rec != nullptr;
#define PT_CASE(P) case P: return launchTrace<P>(count, cont, a, grid, block, s);
    switch (prog) {
        PT_WALK_PROGS(PT_CASE)
    default: return hipErrorInvalidValue;
    }
#undef PT_CASE
}

hipError_t PT_CAT(pt_launch_persist_, PT_WALK_NAME)(int prog, int count, const pt::TraceArgs* a, const pt::WfBufs* w,
                                                    int tiles_x, unsigned n_wave_tiles, unsigned per_wave,
                                                    unsigned refill, dim3 grid, dim3 block, hipStream_t s)
{
    using namespace pt;
#define PT_CASE(P)                                                                                                       \
    case P:                                                                                                               \
        if (count) hipLaunchKernelGGL((pt::pt_persist<P, true>), grid, block, 0, s, *a, *w, tiles_x, n_wave_tiles, per_wave, refill); \
        else hipLaunchKernelGGL((pt::pt_persist<P, false>), grid, block, 0, s, *a, *w, tiles_x, n_wave_tiles, per_wave, refill); \
        break;
    switch (prog) {
        PT_WALK_PROGS(PT_CASE)
    default: return hipErrorInvalidValue;
    }
#undef PT_CASE
    return hipGetLastError();
}

hipError_t PT_CAT(pt_launch_cont_, PT_WALK_NAME)(int prog, const pt::TraceArgs* a, dim3 grid, hipStream_t s)
{
    using namespace pt;
#define PT_CASE(P) case P: return launchCont<P>(a, grid, s);
    switch (prog) {
        PT_WALK_PROGS(PT_CASE)
    default: return hipErrorInvalidValue;
    }
#undef PT_CASE
}
