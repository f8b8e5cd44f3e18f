// obj.hpp — Wavefront OBJ/MTL reader for LoadModelAsPrefab.
//
// The reference reads models with its vendored tinyobjloader 2.x
// (src/core/tiny_obj_loader.h, LoadObj with triangulation, MaterialFileReader
// over the model's directory).  This is a restatement of the parts of that
// reader the importer consumes — positions, normals, texture coordinates,
// faces (triangles; quads split along the shorter diagonal; larger polygons by
// its ear clipping), shape splitting at `o` / `g` and per-face material ids
// from `usemtl` — with tinyobjloader's own number parser, index rules and MTL
// keys (newmtl, Kd, Ke, map_Kd, map_Ke and their texture options), so files
// load to the same arrays.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace pth {

struct obj_index {
    int vertex_index = -1, normal_index = -1, texcoord_index = -1;
};

struct obj_shape {
    std::string name;
    std::vector<obj_index> indices;      // 3 per triangle
    std::vector<int> material_ids;       // 1 per triangle (-1 = none)
};

struct obj_material {
    std::string name;
    float diffuse[3] = {0, 0, 0};
    float emission[3] = {0, 0, 0};
    std::string diffuse_texname;
    std::string emissive_texname;
};

struct obj_data {
    std::vector<float> vertices, normals, texcoords;
    std::vector<obj_shape> shapes;
    std::vector<obj_material> materials;
    std::string warning, error;
};

// LoadObj(attrib, shapes, materials, warn, err, path, mtl_basedir) with
// triangulate = true.  Returns false on an unreadable file or a malformed
// face (zero / out-of-range relative index), like tinyobjloader.
bool LoadObj(obj_data& Out, const char* Path, const char* MtlBaseDir);

// tinyobjloader's tryParseDouble (exposed for tests).
bool ObjParseDouble(const char* s, const char* s_end, double* result);

}  // namespace pth
