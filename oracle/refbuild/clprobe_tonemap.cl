// TEST INFRASTRUCTURE ONLY (oracle/refbuild): the reference's Reinhard tone-mapping functions
// (ToneMapping.cl:32-40 toneMapControlled, colors.cl:19-22 computeLuminanceFromRGB), evaluated on
// the GPU per pixel of a float4 buffer in the order ReinhardToneMapping (ToneMapping.cl:42-63)
// applies them.  The kernel itself reads and writes image2d_t objects, which this GPU's OpenCL
// cannot run, so the probe feeds the same functions from a buffer; the one line of the kernel
// body between them (rgba.xyz *= tL / L) is restated here.  Compiled from the reference sources
// where they lie (-I assets/kernels; the image kernels in the file are compiled, never launched).
// Compared with the product's k_tonemap by tests/test_gpu_postprocess.py.
#include "ToneMapping.cl"

__kernel void ProbeToneMap(__global const float4* in, int n, float Lwhite, __global float4* out)
{
    int i = get_global_id(0);
    if (i >= n) return;
    float4 rgba = in[i];
    float L = computeLuminanceFromRGB(rgba.xyz);
    float tL = toneMapControlled(L, Lwhite);
    rgba.xyz *= tL / L;
    out[i] = rgba;
}
