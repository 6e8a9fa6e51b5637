// pt_trace_walk_quad.hip — the megakernel / persistent kernels of the quad variants: two-level records.
#define PT_WALK_NAME quad
#define PT_WALK_PROGS PT_FOR_EACH_PROG_QUAD
#include "pt_trace_inst.h"
