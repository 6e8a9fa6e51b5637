// pt_trace_walk_trail.hip — the megakernel / persistent kernels of the trail variants: child-pair records, restart trail.
#define PT_WALK_NAME trail
#define PT_WALK_PROGS PT_FOR_EACH_PROG_TRAIL
#include "pt_trace_inst.h"
