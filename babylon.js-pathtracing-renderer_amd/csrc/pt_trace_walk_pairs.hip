// pt_trace_walk_pairs.hip — the megakernel / persistent kernels of the pairs variants: child-pair records, short stack.
#define PT_WALK_NAME pairs
#define PT_WALK_PROGS PT_FOR_EACH_PROG_PAIRS
#include "pt_trace_inst.h"
