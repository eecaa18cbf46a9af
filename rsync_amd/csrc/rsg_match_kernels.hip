// rsg_match_kernels.hip -- sender kernels (filled in next).
#include "rsg_internal.h"
