// scl_kernel.hip -- placeholder, replaced by the SC-list kernel.
#include <hip/hip_runtime.h>
#include "../../../include/polar_mi355x.h"
#include "plan.h"
namespace pl {
size_t scl_workspace_size(const pl_plan*, int64_t) { return 0; }
int launch_scl(const pl_plan*, const float*, int64_t, void*, int, double*, void*, size_t, hipStream_t) {
    set_error("SCL decode not built yet");
    return PL_ENOTSUP;
}
}  // namespace pl
