// hs_kernels_f32.hip -- the same kernels in single precision (BASELINE configs[2]:
// spider, 16384 rollouts x horizon 32, fp32). All arithmetic, LDS and outputs in
// float; topology and gait parameters are converted on load.
#define HS_REAL float
#define HS_REAL_IS_FLOAT 1
#include "hs_kernels.hip"
