// obj.cpp — restatement of the vendored tinyobjloader 2.x reader
// (src/core/tiny_obj_loader.h) for LoadModelAsPrefab; line references are to
// that header.  real_t is float there, so parsed values are narrowed from
// double exactly as it does.
#include "obj.hpp"

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <limits>
#include <map>
#include <sstream>

namespace pth {

namespace {

inline bool IsSpace(char x) { return x == ' ' || x == '\t'; }                 // :801
inline bool IsDigit(char x) { return (unsigned)(x - '0') < 10u; }             // :802
inline bool IsNewLine(char x) { return x == '\r' || x == '\n' || x == '\0'; } // :804

// safeGetline (:767-799): '\n', '\r' or "\r\n" ends a line.
bool GetLine(std::istream& is, std::string& t)
{
    t.clear();
    std::streambuf* sb = is.rdbuf();
    bool any = false;
    for (;;) {
        int c = sb->sbumpc();
        if (c == '\n') return true;
        if (c == '\r') {
            if (sb->sgetc() == '\n') sb->sbumpc();
            return true;
        }
        if (c == EOF) return any;
        t += (char)c;
        any = true;
    }
}

bool FixIndex(int idx, int n, int* ret, bool allow_zero)                      // :819-851
{
    if (idx > 0) { *ret = idx - 1; return true; }
    if (idx == 0) { *ret = idx - 1; return allow_zero; }
    *ret = n + idx;
    return *ret >= 0;
}

std::string ParseString(const char** token)                                   // :854-861
{
    (*token) += strspn(*token, " \t");
    size_t e = strcspn(*token, " \t\r");
    std::string s(*token, *token + e);
    (*token) += e;
    return s;
}

float ParseReal(const char** token, double default_value = 0.0)               // :1030-1038
{
    (*token) += strspn(*token, " \t");
    const char* end = *token + strcspn(*token, " \t\r");
    double val = default_value;
    ObjParseDouble(*token, end, &val);
    *token = end;
    return (float)val;
}

bool ParseReal(const char** token, float* out)                                // :1040-1051
{
    (*token) += strspn(*token, " \t");
    const char* end = *token + strcspn(*token, " \t\r");
    double val;
    bool ok = ObjParseDouble(*token, end, &val);
    if (ok) *out = (float)val;
    *token = end;
    return ok;
}

void ParseOnOff(const char** token)                                           // parseOnOff: consumes one token
{
    (*token) += strspn(*token, " \t");
    (*token) += strcspn(*token, " \t\r");
}

struct vertex_index { int v = -1, vt = -1, vn = -1; };

bool ParseTriple(const char** token, int vsize, int vnsize, int vtsize, vertex_index* ret)   // :1188-1236
{
    vertex_index vi;
    if (!FixIndex(atoi(*token), vsize, &vi.v, false)) return false;
    (*token) += strcspn(*token, "/ \t\r");
    if ((*token)[0] != '/') { *ret = vi; return true; }
    (*token)++;
    if ((*token)[0] == '/') {
        (*token)++;
        if (!FixIndex(atoi(*token), vnsize, &vi.vn, true)) return false;
        (*token) += strcspn(*token, "/ \t\r");
        *ret = vi;
        return true;
    }
    if (!FixIndex(atoi(*token), vtsize, &vi.vt, true)) return false;
    (*token) += strcspn(*token, "/ \t\r");
    if ((*token)[0] != '/') { *ret = vi; return true; }
    (*token)++;
    if (!FixIndex(atoi(*token), vnsize, &vi.vn, true)) return false;
    (*token) += strcspn(*token, "/ \t\r");
    *ret = vi;
    return true;
}

// ParseTextureNameAndOption (:1274-1355): options are skipped with the same
// token consumption; the name is the remainder of the line.
void ParseTextureName(std::string* texname, const char* token)
{
    bool found = false;
    std::string name;
    while (!IsNewLine(*token)) {
        token += strspn(token, " \t");
        auto opt = [&](const char* o) {
            size_t n = strlen(o);
            return strncmp(token, o, n) == 0 && IsSpace(token[n]);
        };
        if (opt("-blendu") || opt("-blendv")) { token += 8; ParseOnOff(&token); }
        else if (opt("-clamp")) { token += 7; ParseOnOff(&token); }
        else if (opt("-boost")) { token += 7; ParseReal(&token, 1.0); }
        else if (opt("-bm")) { token += 4; ParseReal(&token, 1.0); }
        else if (opt("-o") || opt("-t")) { token += 3; ParseReal(&token); ParseReal(&token); ParseReal(&token); }
        else if (opt("-s")) { token += 3; ParseReal(&token, 1.0); ParseReal(&token, 1.0); ParseReal(&token, 1.0); }
        else if (opt("-type")) { token += 5; ParseString(&token); }
        else if (opt("-texres")) {
            token += 7;
            token += strspn(token, " \t");
            token += strcspn(token, " \t\r");
        } else if (opt("-imfchan")) {
            token += 9;
            token += strspn(token, " \t");
            token += strcspn(token, " \t\r");
        } else if (opt("-mm")) { token += 4; ParseReal(&token, 0.0); ParseReal(&token, 1.0); }
        else if (opt("-colorspace")) { token += 12; ParseString(&token); }
        else {
            name = std::string(token);
            token += name.length();
            found = true;
        }
    }
    if (found) *texname = name;
}

// LoadMtl (:2069-2466), the keys the importer reads.
void LoadMtl(std::map<std::string, int>& material_map, std::vector<obj_material>& materials, std::istream& in)
{
    obj_material material;
    bool has_kd = false;   // not reset by newmtl (:2130-2136)
    std::string linebuf;
    while (in.peek() != -1) {
        GetLine(in, linebuf);
        if (!linebuf.empty()) linebuf = linebuf.substr(0, linebuf.find_last_not_of(" \t") + 1);
        if (!linebuf.empty() && linebuf.back() == '\n') linebuf.pop_back();
        if (!linebuf.empty() && linebuf.back() == '\r') linebuf.pop_back();
        if (linebuf.empty()) continue;
        const char* token = linebuf.c_str();
        token += strspn(token, " \t");
        if (token[0] == '\0' || token[0] == '#') continue;
        if (strncmp(token, "newmtl", 6) == 0 && IsSpace(token[6])) {
            if (!material.name.empty()) {
                material_map.insert({material.name, (int)materials.size()});
                materials.push_back(material);
            }
            material = obj_material();
            token += 7;
            material.name = ParseString(&token);
            continue;
        }
        if (token[0] == 'K' && token[1] == 'd' && IsSpace(token[2])) {
            token += 2;
            for (int i = 0; i < 3; i++) material.diffuse[i] = ParseReal(&token);
            has_kd = true;
            continue;
        }
        if (token[0] == 'K' && token[1] == 'e' && IsSpace(token[2])) {
            token += 2;
            for (int i = 0; i < 3; i++) material.emission[i] = ParseReal(&token);
            continue;
        }
        if (strncmp(token, "map_Kd", 6) == 0 && IsSpace(token[6])) {
            token += 7;
            ParseTextureName(&material.diffuse_texname, token);
            if (!has_kd) material.diffuse[0] = material.diffuse[1] = material.diffuse[2] = 0.6f;
            continue;
        }
        if (strncmp(token, "map_Ke", 6) == 0 && IsSpace(token[6])) {
            token += 7;
            ParseTextureName(&material.emissive_texname, token);
            continue;
        }
        // every other statement leaves these fields unchanged
    }
    material_map.insert({material.name, (int)materials.size()});
    materials.push_back(material);
}

struct face { std::vector<vertex_index> v; };

struct prim_group {
    std::vector<face> faces;
    size_t line_indices = 0, point_indices = 0;   // only their presence matters here
    bool lines = false, points = false;
    bool IsEmpty() const { return faces.empty() && !lines && !points; }
};

struct shape_acc {
    obj_shape s;
    size_t line_indices = 0, point_indices = 0;
};

int PointInTriangle(const float* vx, const float* vy, float tx, float ty)   // pnpoly (:1440-1450), nvert = 3
{
    int c = 0;
    for (int i = 0, j = 2; i < 3; j = i++)
        if (((vy[i] > ty) != (vy[j] > ty)) && (tx < (vx[j] - vx[i]) * (ty - vy[i]) / (vy[j] - vy[i]) + vx[i])) c = !c;
    return c;
}

void PushTri(obj_shape& s, const vertex_index& a, const vertex_index& b, const vertex_index& c, int material)
{
    for (const vertex_index* p : {&a, &b, &c}) {
        obj_index i;
        i.vertex_index = p->v;
        i.normal_index = p->vn;
        i.texcoord_index = p->vt;
        s.indices.push_back(i);
    }
    s.material_ids.push_back(material);
}

// exportGroupsToShape (:1482-1990) with triangulate = true, built-in ear clipping.
bool ExportGroups(shape_acc& shape, const prim_group& g, int material, const std::string& name,
                  const std::vector<float>& v)
{
    if (g.IsEmpty()) return false;
    shape.s.name = name;
    for (const face& f : g.faces) {
        size_t npolys = f.v.size();
        if (npolys < 3) continue;
        if (npolys == 3) {
            PushTri(shape.s, f.v[0], f.v[1], f.v[2], material);
            continue;
        }
        if (npolys == 4) {
            const vertex_index &i0 = f.v[0], &i1 = f.v[1], &i2 = f.v[2], &i3 = f.v[3];
            size_t vi0 = (size_t)i0.v, vi1 = (size_t)i1.v, vi2 = (size_t)i2.v, vi3 = (size_t)i3.v;
            if (3 * vi0 + 2 >= v.size() || 3 * vi1 + 2 >= v.size() || 3 * vi2 + 2 >= v.size() ||
                3 * vi3 + 2 >= v.size())
                continue;
            float e02x = v[vi2 * 3 + 0] - v[vi0 * 3 + 0], e02y = v[vi2 * 3 + 1] - v[vi0 * 3 + 1],
                  e02z = v[vi2 * 3 + 2] - v[vi0 * 3 + 2];
            float e13x = v[vi3 * 3 + 0] - v[vi1 * 3 + 0], e13y = v[vi3 * 3 + 1] - v[vi1 * 3 + 1],
                  e13z = v[vi3 * 3 + 2] - v[vi1 * 3 + 2];
            float sqr02 = e02x * e02x + e02y * e02y + e02z * e02z;
            float sqr13 = e13x * e13x + e13y * e13y + e13z * e13z;
            if (sqr02 < sqr13) {
                PushTri(shape.s, i0, i1, i2, material);
                PushTri(shape.s, i0, i2, i3, material);
            } else {
                PushTri(shape.s, i0, i1, i3, material);
                PushTri(shape.s, i1, i2, i3, material);
            }
            continue;
        }
        // Ear clipping (:1741-1947): projection axes from the first
        // non-degenerate corner, then clip ears in polygon order.
        size_t axes[2] = {1, 2};
        for (size_t k = 0; k < npolys; ++k) {
            size_t vi0 = (size_t)f.v[(k + 0) % npolys].v, vi1 = (size_t)f.v[(k + 1) % npolys].v,
                   vi2 = (size_t)f.v[(k + 2) % npolys].v;
            if (3 * vi0 + 2 >= v.size() || 3 * vi1 + 2 >= v.size() || 3 * vi2 + 2 >= v.size()) continue;
            float e0x = v[vi1 * 3 + 0] - v[vi0 * 3 + 0], e0y = v[vi1 * 3 + 1] - v[vi0 * 3 + 1],
                  e0z = v[vi1 * 3 + 2] - v[vi0 * 3 + 2];
            float e1x = v[vi2 * 3 + 0] - v[vi1 * 3 + 0], e1y = v[vi2 * 3 + 1] - v[vi1 * 3 + 1],
                  e1z = v[vi2 * 3 + 2] - v[vi1 * 3 + 2];
            float cx = std::fabs(e0y * e1z - e0z * e1y);
            float cy = std::fabs(e0z * e1x - e0x * e1z);
            float cz = std::fabs(e0x * e1y - e0y * e1x);
            const float eps = std::numeric_limits<float>::epsilon();
            if (cx > eps || cy > eps || cz > eps) {
                if (!(cx > cy && cx > cz)) {
                    axes[0] = 0;
                    if (cz > cx && cz > cy) axes[1] = 1;
                }
                break;
            }
        }
        std::vector<vertex_index> rem = f.v;
        size_t guess_vert = 0;
        vertex_index ind[3];
        float vx[3], vy[3];
        size_t remainingIterations = f.v.size();
        size_t previousRemaining = rem.size();
        while (rem.size() > 3 && remainingIterations > 0) {
            npolys = rem.size();
            if (guess_vert >= npolys) guess_vert -= npolys;
            if (previousRemaining != npolys) {
                previousRemaining = npolys;
                remainingIterations = npolys;
            } else {
                remainingIterations--;
            }
            for (size_t k = 0; k < 3; k++) {
                ind[k] = rem[(guess_vert + k) % npolys];
                size_t vi = (size_t)ind[k].v;
                if (vi * 3 + axes[0] >= v.size() || vi * 3 + axes[1] >= v.size()) {
                    vx[k] = 0.0f;
                    vy[k] = 0.0f;
                } else {
                    vx[k] = v[vi * 3 + axes[0]];
                    vy[k] = v[vi * 3 + axes[1]];
                }
            }
            float e0x = vx[1] - vx[0], e0y = vy[1] - vy[0];
            float e1x = vx[2] - vx[1], e1y = vy[2] - vy[1];
            float cross = e0x * e1y - e0y * e1x;
            float area = (vx[0] * vy[1] - vy[0] * vx[1]) * 0.5f;
            if (cross * area < 0.0f) {
                guess_vert += 1;
                continue;
            }
            bool overlap = false;
            for (size_t other = 3; other < npolys; ++other) {
                size_t idx = (guess_vert + other) % npolys;
                if (idx >= rem.size()) continue;
                size_t ovi = (size_t)rem[idx].v;
                if (ovi * 3 + axes[0] >= v.size() || ovi * 3 + axes[1] >= v.size()) continue;
                if (PointInTriangle(vx, vy, v[ovi * 3 + axes[0]], v[ovi * 3 + axes[1]])) {
                    overlap = true;
                    break;
                }
            }
            if (overlap) {
                guess_vert += 1;
                continue;
            }
            PushTri(shape.s, ind[0], ind[1], ind[2], material);
            size_t removed = (guess_vert + 1) % npolys;
            while (removed + 1 < npolys) {
                rem[removed] = rem[removed + 1];
                removed += 1;
            }
            rem.pop_back();
        }
        if (rem.size() == 3) PushTri(shape.s, rem[0], rem[1], rem[2], material);
    }
    if (g.lines) shape.line_indices += g.line_indices;
    if (g.points) shape.point_indices += g.point_indices;
    return true;
}

// SplitString (:2008-2040) on ' ' with '\\' escapes.
std::vector<std::string> SplitString(const std::string& s, char delim, char escape)
{
    std::vector<std::string> elems;
    std::string token;
    bool escaping = false;
    for (size_t i = 0; i < s.size(); ++i) {
        char ch = s[i];
        if (escaping) {
            escaping = false;
        } else if (ch == escape) {
            escaping = true;
            continue;
        } else if (ch == delim) {
            if (!token.empty()) elems.push_back(token);
            token.clear();
            continue;
        }
        token += ch;
    }
    elems.push_back(token);
    return elems;
}

}  // namespace

bool ObjParseDouble(const char* s, const char* s_end, double* result)         // tryParseDouble (:897-1028)
{
    if (s >= s_end) return false;
    double mantissa = 0.0;
    int exponent = 0;
    char sign = '+', exp_sign = '+';
    const char* curr = s;
    int read = 0;
    bool end_not_reached = false;
    bool leading_decimal_dots = false;

    if (*curr == '+' || *curr == '-') {
        sign = *curr;
        curr++;
        if (curr != s_end && *curr == '.') leading_decimal_dots = true;
    } else if (IsDigit(*curr)) {
    } else if (*curr == '.') {
        leading_decimal_dots = true;
    } else {
        return false;
    }
    end_not_reached = curr != s_end;
    if (!leading_decimal_dots) {
        while (end_not_reached && IsDigit(*curr)) {
            mantissa *= 10;
            mantissa += (int)(*curr - 0x30);
            curr++;
            read++;
            end_not_reached = curr != s_end;
        }
        if (read == 0) return false;
    }
    if (!end_not_reached) goto assemble;
    if (*curr == '.') {
        curr++;
        read = 1;
        end_not_reached = curr != s_end;
        while (end_not_reached && IsDigit(*curr)) {
            static const double pow_lut[] = {1.0, 0.1, 0.01, 0.001, 0.0001, 0.00001, 0.000001, 0.0000001};
            const int lut_entries = sizeof pow_lut / sizeof pow_lut[0];
            mantissa += (int)(*curr - 0x30) * (read < lut_entries ? pow_lut[read] : std::pow(10.0, -read));
            read++;
            curr++;
            end_not_reached = curr != s_end;
        }
    } else if (*curr == 'e' || *curr == 'E') {
    } else {
        goto assemble;
    }
    if (!end_not_reached) goto assemble;
    if (*curr == 'e' || *curr == 'E') {
        curr++;
        end_not_reached = curr != s_end;
        if (end_not_reached && (*curr == '+' || *curr == '-')) {
            exp_sign = *curr;
            curr++;
        } else if (IsDigit(*curr)) {
        } else {
            return false;
        }
        read = 0;
        end_not_reached = curr != s_end;
        while (end_not_reached && IsDigit(*curr)) {
            if (exponent > (2147483647 / 10)) return false;
            exponent *= 10;
            exponent += (int)(*curr - 0x30);
            curr++;
            read++;
            end_not_reached = curr != s_end;
        }
        exponent *= (exp_sign == '+' ? 1 : -1);
        if (read == 0) return false;
    }
assemble:
    *result = (sign == '+' ? 1 : -1) * (exponent ? std::ldexp(mantissa * std::pow(5.0, exponent), exponent) : mantissa);
    return true;
}

bool LoadObj(obj_data& Out, const char* Path, const char* MtlBaseDir)          // :2547-2583, :2585-3150
{
    Out = obj_data();
    std::ifstream ifs(Path);
    if (!ifs) {
        Out.error = std::string("Cannot open file [") + Path + "]\n";
        return false;
    }
    std::string baseDir = MtlBaseDir ? MtlBaseDir : "";
    if (!baseDir.empty() && baseDir.back() != '/') baseDir += '/';

    std::vector<float>& v = Out.vertices;
    std::vector<float>& vn = Out.normals;
    std::vector<float>& vt = Out.texcoords;
    std::map<std::string, int> material_map;
    std::vector<std::string> loaded_mtl;
    prim_group group;
    std::string name;
    int material = -1;
    shape_acc shape;

    auto push_shape = [&](bool cond) {
        if (cond) Out.shapes.push_back(shape.s);
    };

    std::string linebuf;
    size_t line_num = 0;
    while (ifs.peek() != -1) {
        GetLine(ifs, linebuf);
        line_num++;
        if (!linebuf.empty() && linebuf.back() == '\n') linebuf.pop_back();
        if (!linebuf.empty() && linebuf.back() == '\r') linebuf.pop_back();
        if (linebuf.empty()) continue;
        const char* token = linebuf.c_str();
        token += strspn(token, " \t");
        if (token[0] == '\0' || token[0] == '#') continue;

        if (token[0] == 'v' && IsSpace(token[1])) {                              // parseVertexWithColor
            token += 2;
            float x = ParseReal(&token), y = ParseReal(&token), z = ParseReal(&token);
            v.push_back(x);
            v.push_back(y);
            v.push_back(z);
            continue;
        }
        if (token[0] == 'v' && token[1] == 'n' && IsSpace(token[2])) {
            token += 3;
            float x = ParseReal(&token), y = ParseReal(&token), z = ParseReal(&token);
            vn.push_back(x);
            vn.push_back(y);
            vn.push_back(z);
            continue;
        }
        if (token[0] == 'v' && token[1] == 't' && IsSpace(token[2])) {
            token += 3;
            float x = ParseReal(&token), y = ParseReal(&token);
            vt.push_back(x);
            vt.push_back(y);
            continue;
        }
        if (token[0] == 'v' && token[1] == 'w' && IsSpace(token[2])) continue;
        if ((token[0] == 'l' || token[0] == 'p') && IsSpace(token[1])) {
            bool is_line = token[0] == 'l';
            token += 2;
            size_t count = 0;
            while (!IsNewLine(token[0])) {
                vertex_index vi;
                if (!ParseTriple(&token, (int)(v.size() / 3), (int)(vn.size() / 3), (int)(vt.size() / 2), &vi)) {
                    Out.error += "Failed to parse `l'/`p' line " + std::to_string(line_num) + "\n";
                    return false;
                }
                count++;
                token += strspn(token, " \t\r");
            }
            if (is_line) { group.lines = true; group.line_indices += count; }
            else { group.points = true; group.point_indices += count; }
            continue;
        }
        if (token[0] == 'f' && IsSpace(token[1])) {
            token += 2;
            token += strspn(token, " \t");
            face f;
            while (!IsNewLine(token[0])) {
                vertex_index vi;
                if (!ParseTriple(&token, (int)(v.size() / 3), (int)(vn.size() / 3), (int)(vt.size() / 2), &vi)) {
                    Out.error += "Failed to parse `f' line (e.g. a zero value for vertex index or invalid relative "
                                 "vertex index). Line " + std::to_string(line_num) + ").\n";
                    return false;
                }
                f.v.push_back(vi);
                token += strspn(token, " \t\r");
            }
            group.faces.push_back(f);
            continue;
        }
        if (strncmp(token, "usemtl", 6) == 0) {
            token += 6;
            std::string namebuf = ParseString(&token);
            int newMaterialId = -1;
            auto it = material_map.find(namebuf);
            if (it != material_map.end()) newMaterialId = it->second;
            else Out.warning += "material [ '" + namebuf + "' ] not found in .mtl\n";
            if (newMaterialId != material) {
                ExportGroups(shape, group, material, name, v);
                group.faces.clear();
                material = newMaterialId;
            }
            continue;
        }
        if (strncmp(token, "mtllib", 6) == 0 && IsSpace(token[6])) {
            token += 7;
            std::vector<std::string> files = SplitString(std::string(token), ' ', '\\');
            bool found = false;
            for (const std::string& fn : files) {
                bool seen = false;
                for (const std::string& l : loaded_mtl) seen |= l == fn;
                if (seen) { found = true; continue; }
                // MaterialFileReader (:2469-2524): every ':'-separated base path
                std::vector<std::string> paths;
                if (baseDir.empty()) {
                    paths.push_back("");
                } else {
                    std::istringstream bs(baseDir);
                    std::string p;
                    while (std::getline(bs, p, ':')) paths.push_back(p);
                }
                bool ok = false;
                for (const std::string& p : paths) {
                    std::string path = p.empty() ? fn : (p.back() == '/' ? p + fn : p + "/" + fn);
                    std::ifstream m(path);
                    if (m) {
                        LoadMtl(material_map, Out.materials, m);
                        ok = true;
                        break;
                    }
                }
                if (ok) {
                    loaded_mtl.push_back(fn);
                    found = true;
                    break;
                }
            }
            if (!found) Out.warning += "Failed to load material file(s). Use default material.\n";
            continue;
        }
        if (token[0] == 'g' && IsSpace(token[1])) {
            ExportGroups(shape, group, material, name, v);
            push_shape(!shape.s.indices.empty());
            shape = shape_acc();
            group = prim_group();
            std::vector<std::string> names;
            while (!IsNewLine(token[0])) {
                names.push_back(ParseString(&token));
                token += strspn(token, " \t\r");
            }
            if (names.size() < 2) {
                name = "";
            } else {
                std::string n = names[1];
                for (size_t i = 2; i < names.size(); i++) n += " " + names[i];
                name = n;
            }
            continue;
        }
        if (token[0] == 'o' && IsSpace(token[1])) {
            ExportGroups(shape, group, material, name, v);
            push_shape(!shape.s.indices.empty() || shape.line_indices > 0 || shape.point_indices > 0);
            group = prim_group();
            shape = shape_acc();
            token += 2;
            name = std::string(token);
            continue;
        }
        // 't' (tags), 's' (smoothing groups) and unknown statements carry
        // nothing the importer reads.
    }
    bool ret = ExportGroups(shape, group, material, name, v);
    push_shape(ret || !shape.s.indices.empty());
    return true;
}

}  // namespace pth
