// Shared helpers of the compiled C ABI consumers (capi_consumer.cpp, capi_rccl.cpp): status
// checks in the shape of INTEGRATION.md's MCRTBridge.h, raw-array I/O, and the scene directory
// written by tests/test_gpu_capi_consumer.py (RTScene::setSceneArgs's 15 arrays + a camera).
#pragma once
#include <hip/hip_runtime.h>

#include <fstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "mcrt_capi.h"

namespace consumer {

inline void check(mcrt_status s, mcrt_ctx c) {
    if (s != MCRT_OK) throw std::runtime_error(mcrt_last_error(c));
}
inline void hipCheck(hipError_t e) {
    if (e != hipSuccess) throw std::runtime_error(hipGetErrorString(e));
}

template <class T>
std::vector<T> load(const std::string& path) {
    std::ifstream f(path, std::ios::binary | std::ios::ate);
    if (!f) return {};
    const size_t n = (size_t)f.tellg();
    std::vector<T> v(n / sizeof(T));
    f.seekg(0);
    f.read(reinterpret_cast<char*>(v.data()), (std::streamsize)(v.size() * sizeof(T)));
    return v;
}
template <class T>
void save(const std::string& path, const T* p, size_t n) {
    std::ofstream f(path, std::ios::binary);
    f.write(reinterpret_cast<const char*>(p), (std::streamsize)(n * sizeof(T)));
}

// The host arrays of one scene directory; desc() points into them (RTScene::commit's inputs).
struct SceneFiles {
    std::vector<mcrt_shape> shapes;
    std::vector<uint32_t> indices;
    std::vector<mcrt_float4> positions, normals, tangents, binormals;
    std::vector<mcrt_float2> uvs;
    std::vector<mcrt_texture_desc> textures;
    std::vector<uint8_t> texData;
    std::vector<uint32_t> sobol;
    std::vector<mcrt_light> lights;
    std::vector<mcrt_material> materials;
    std::vector<mcrt_camera> camera;

    explicit SceneFiles(const std::string& in) {
        shapes = load<mcrt_shape>(in + "/shapes.bin");
        indices = load<uint32_t>(in + "/indices.bin");
        positions = load<mcrt_float4>(in + "/positions.bin");
        uvs = load<mcrt_float2>(in + "/uvs.bin");
        normals = load<mcrt_float4>(in + "/normals.bin");
        tangents = load<mcrt_float4>(in + "/tangents.bin");
        binormals = load<mcrt_float4>(in + "/binormals.bin");
        textures = load<mcrt_texture_desc>(in + "/textures.bin");
        texData = load<uint8_t>(in + "/texdata.bin");
        sobol = load<uint32_t>(in + "/sobol.bin");
        lights = load<mcrt_light>(in + "/lights.bin");
        materials = load<mcrt_material>(in + "/materials.bin");
        camera = load<mcrt_camera>(in + "/camera.bin");
    }
    mcrt_scene_desc desc() const {
        mcrt_scene_desc d = {};
        d.shapes = shapes.data();                 d.num_shapes = (uint32_t)shapes.size();
        d.indices = indices.data();               d.num_indices = (uint32_t)indices.size();
        d.positions = positions.data();           d.num_vertices = (uint32_t)positions.size();
        d.uvs = uvs.data();
        d.normals = normals.data();
        d.tangents = tangents.data();
        d.binormals = binormals.data();
        d.textures = textures.data();             d.num_textures = (uint32_t)textures.size();
        d.tex_data = texData.data();              d.tex_data_bytes = texData.size();
        d.sobol_matrices = sobol.data();          d.num_sobol_words = (uint32_t)sobol.size();
        d.lights = lights.data();                 d.num_lights = (uint32_t)lights.size();
        d.materials = materials.data();           d.num_materials = (uint32_t)materials.size();
        return d;
    }
};

}  // namespace consumer
