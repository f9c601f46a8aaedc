// TEST INFRASTRUCTURE ONLY (oracle/refbuild): the reference's reconstruction filter weights
// (filters.cl:12-69, selected exactly as ReconstructionPass does, reconstruction.cl:21-42),
// evaluated on the GPU for a list of RTFilterProperties with the DEVICE layout of
// kernel_data.h:63-80 (56 B; the reference host writes a 48-B struct, SURVEY App. A Q9, which this
// probe does not reproduce -- it pins the filter functions themselves).  Compiled from the
// reference sources where they lie (-I assets/kernels).  Compared with the product's k_accumulate
// weights by tests/test_gpu_accumulate.py.
#include "kernel_data.h"
#include "filters.cl"

__kernel void ProbeFilters(__global const RTFilterProperties* filterProperties, int n, __global float* out)
{
    int i = get_global_id(0);
    if (i >= n) return;
    __global const RTFilterProperties* fp = filterProperties + i;
    float filterWeight;
    switch (fp->filterType)
    {
    case RT_BOX_FILTER:
        filterWeight = 1.0f;
        break;
    case RT_TRIANGLE_FILTER:
        filterWeight = evaluateTriangleFilter(fp->pixelOffset, fp->radius);
        break;
    case RT_GAUSSIAN_FILTER:
        filterWeight = evaluateGaussianFilter(fp->pixelOffset, fp->gaussianAlpha, fp->gaussianExpX, fp->gaussianExpY);
        break;
    case RT_MITCHELL_FILTER:
        filterWeight = evaluateMitchellFilter(fp->pixelOffset, fp->radius, fp->mitchellB, fp->mitchellC);
        break;
    case RT_LANCZOS_SINC_FILTER:
        filterWeight = evaluateLanczosFilter(fp->pixelOffset, fp->radius, fp->lanczosSincTau);
        break;
    }
    out[i] = filterWeight;
}
