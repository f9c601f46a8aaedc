// TEST INFRASTRUCTURE ONLY (oracle/refbuild): probe over the reference's own texture-LOD
// functions, which its PathTracing kernel carries but never calls (textures.cl:204-209), compiled
// from the reference sources where they lie (-I assets/kernels).  Per pixel, from the reference's
// own primary RTIntersection and RTRayDifferentials (GeneratePerspectiveRays, PathTracing.cl:13-35):
//   out[3i+0] = (si.duvdx, si.duvdy)      computeSurfaceInteractionWithDifferentials (geometry.cl:92-175)
//   out[3i+1] = (lod, shapeid bits, si.uv) computeMipmapLOD (textures.cl:198-202) of the diffuse texture
//   out[3i+2] = readTexture2Df_lod(diffuse texture, si.uv, lod) (textures.cl:148-196)
// Compared with the product's MCRT_AOV_TEXTURE_LOD output by tests/test_gpu_texture_lod.py.
#include "PathTracing.cl"

__kernel void ProbeLOD(SCENE_PARAMS, int image_width, int image_height,
                       __global const RTIntersection* isects, __global const RTRayDifferentials* diffs,
                       __global float4* out)
{
    int i = get_global_id(0);
    if (i >= image_width * image_height) return;
    MAKE_SCENE(scene);
    RTIntersection isect = isects[i];
    __global float4* o = out + 3 * i;
    if (isect.shapeid == -1 || isect.primid == -1) return;
    RTInteraction si = computeSurfaceInteractionWithDifferentials(&scene, &isect, diffs + i);
    int materialId = scene_shapes[isect.shapeid].materialId;
    float lod = 0.0f;
    float4 c = (float4)(0.0f);
    if (materialId != RT_INVALID_ID && scene_materials[materialId].uber_diffuseTexId != RT_INVALID_ID)
    {
        TextureDesc2D desc = scene_textures2D[scene_materials[materialId].uber_diffuseTexId];
        lod = computeMipmapLOD(&desc, si.duvdx, si.duvdy);
        c = readTexture2Df_lod(&desc, scene_texData2D, si.uv, lod);
    }
    o[0] = (float4)(si.duvdx, si.duvdy);
    o[1] = (float4)(lod, as_float(isect.shapeid), si.uv);
    o[2] = c;
}
