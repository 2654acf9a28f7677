// MFMA implicit-GEMM kernels for the Nature-CNN dueling network.
// (filled in by the conv milestone; this translation unit is part of the library build)
#include "common.h"
#include "kernels.h"

namespace apex {}  // namespace apex
