// mcg_nested_kernels.hip -- nested sampling kernels (placeholder, filled in next).
#include "mcg_device.h"
