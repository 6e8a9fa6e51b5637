// pt_trace_walk_ref.hip — the megakernel / persistent kernels of the ref variants: the reference's texel walk (and the programs without a mesh).
#define PT_WALK_NAME ref
#define PT_WALK_PROGS PT_FOR_EACH_PROG_REF
#include "pt_trace_inst.h"
