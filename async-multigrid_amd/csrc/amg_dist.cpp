// amg_dist.cpp -- multi-GPU row-slab partition and RCCL halo exchange (placeholder, filled in next).
#include "amg_internal.h"
