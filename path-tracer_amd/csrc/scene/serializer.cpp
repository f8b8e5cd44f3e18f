// serializer.cpp — the scene file format: LoadScene / SaveScene.
//
// Restates src/scene/serializer.cpp (:1-529) of the reference:
//   * <scene>.json: nlohmann::json dump(4) of {"Textures", "Materials",
//     "Meshes", "Prefabs", "Root"} (serializer.cpp:395-479).  Keys are
//     written in nlohmann's default std::map order (sorted), arrays of
//     vec2/vec3/vec4 as JSON arrays, enums as integers, object references
//     (texture / material / mesh pointers) as indices into the scene's
//     vectors with -1 for null (:214-230, :250-266, :318-334);
//   * one <name>.texture per texture: {'TEX ', 0, Width, Height} + the
//     compressed rgba32f pixels (:174-212);
//   * one <name>.mesh per mesh: {'MESH', 0, FaceCount, NodeCount} + the
//     compressed faces and BVH nodes (:269-316);
//   * spectrum.dat: {'SPEC', 0} + the compressed RGB->spectrum coefficient
//     table (:481-509).
// A compressed block is an `mz_ulong` byte count followed by a zlib stream
// (mz_compress / mz_uncompress, :16-44): zlib's compress2 / uncompress read
// and write the same streams.  mz_ulong is `unsigned long`, 4 bytes on the
// reference's platform: its WriteCompressed calls std::max(Size, 1024ull)
// (:18), which only compiles where size_t is unsigned long long, i.e. an
// LLP64 (MSVC x64) build.  So blocks are written with a 4-byte count, and the
// reader also accepts an 8-byte one.  File names come
// from MakeFileName (:46-59): every non-alphanumeric character becomes '_'.
//
// Deliberate differences, each compatible with the reference's reader:
//   * the reference writes no mesh vertices (:287-292), so a scene it
//     reloads has empty vertex arrays.  Here the .mesh file continues after
//     the nodes with a u64 vertex count and a third compressed block holding
//     the vertices (the reference's reader stops after the nodes and ignores
//     them); a file without them loads with no vertices, as in the reference;
//   * the root's SkyboxSamplingProbability (not serialised, :352-359) is
//     written as an extra key and read when present;
//   * two textures (or meshes) whose names map to the same file name
//     overwrite each other's file in the reference (an OBJ shape split by
//     material gives several meshes of one name).  Here a later one gets a
//     numbered file name, recorded under an extra "FileName" key that the
//     reader prefers;
//   * a key missing on read keeps the default instead of throwing, and
//     mesh depth (not serialised) is recomputed from the loaded nodes.
#include "scene.hpp"

#include <zlib.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <filesystem>
#include <fstream>
#include <map>
#include <sstream>
#include <unordered_map>

namespace pth {
namespace {

// --- a small JSON document model (the subset of nlohmann::json used) ---------

struct json {
    enum kind { Null, Boolean, Integer, Unsigned, Float, String, Array, Object };
    kind k = Null;
    bool b = false;
    int64_t i = 0;
    uint64_t u = 0;
    double d = 0;
    std::string s;
    std::vector<json> a;
    std::map<std::string, json> o;

    static json number(double v) { json j; j.k = Float; j.d = v; return j; }
    static json integer(int64_t v) { json j; j.k = Integer; j.i = v; return j; }
    static json uinteger(uint64_t v) { json j; j.k = Unsigned; j.u = v; return j; }
    static json boolean(bool v) { json j; j.k = Boolean; j.b = v; return j; }
    static json string(const std::string& v) { json j; j.k = String; j.s = v; return j; }

    // nlohmann operator[] on a non-const value: null becomes an object/array.
    json& operator[](const std::string& key)
    {
        if (k == Null) k = Object;
        return o[key];
    }
    json& push_back(json v)
    {
        if (k == Null) k = Array;
        a.push_back(std::move(v));
        return a.back();
    }
    const json* find(const std::string& key) const
    {
        if (k != Object) return nullptr;
        auto it = o.find(key);
        return it == o.end() ? nullptr : &it->second;
    }
    size_t size() const { return k == Array ? a.size() : k == Object ? o.size() : k == Null ? 0 : 1; }
    bool is_number() const { return k == Integer || k == Unsigned || k == Float; }
    double num() const { return k == Integer ? (double)i : k == Unsigned ? (double)u : k == Float ? d : 0.0; }
    int64_t inum() const { return k == Integer ? i : k == Unsigned ? (int64_t)u : k == Float ? (int64_t)d : 0; }
};

// nlohmann::detail::serializer::dump_escaped with ensure_ascii = false.
void DumpString(std::string& out, const std::string& s)
{
    out += '"';
    for (unsigned char c : s) {
        switch (c) {
            case '"': out += "\\\""; break;
            case '\\': out += "\\\\"; break;
            case '\b': out += "\\b"; break;
            case '\f': out += "\\f"; break;
            case '\n': out += "\\n"; break;
            case '\r': out += "\\r"; break;
            case '\t': out += "\\t"; break;
            default:
                if (c < 0x20) {
                    char buf[8];
                    std::snprintf(buf, sizeof buf, "\\u%04x", c);
                    out += buf;
                } else {
                    out += (char)c;
                }
        }
    }
    out += '"';
}

// Shortest round-trip decimal digits of a double, laid out like nlohmann's
// to_chars / format_buffer (min_exp -4, max_exp 15): "1.0", "0.001",
// "1.5e-05", "1e+16".
void DumpFloat(std::string& out, double v)
{
    if (!std::isfinite(v)) { out += "null"; return; }
    if (v == 0) { out += std::signbit(v) ? "-0.0" : "0.0"; return; }
    char buf[40];
    int prec = 1;
    for (; prec <= 17; prec++) {
        std::snprintf(buf, sizeof buf, "%.*e", prec - 1, v);
        if (std::strtod(buf, nullptr) == v) break;
    }
    // buf = [-]d.ddde[+-]XX: split into digits and decimal exponent.
    std::string str(buf);
    bool neg = str[0] == '-';
    if (neg) str = str.substr(1);
    size_t epos = str.find('e');
    int e10 = std::atoi(str.c_str() + epos + 1);
    std::string digits;
    for (size_t p = 0; p < epos; p++)
        if (str[p] != '.') digits += str[p];
    while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
    int k = (int)digits.size();
    int n = e10 + 1;   // position of the decimal point relative to the digits
    std::string r;
    if (k <= n && n <= 15) {
        r = digits + std::string(n - k, '0') + ".0";
    } else if (0 < n && n <= 15) {
        r = digits.substr(0, n) + "." + digits.substr(n);
    } else if (-4 < n && n <= 0) {
        r = "0." + std::string(-n, '0') + digits;
    } else {
        r = digits.substr(0, 1);
        if (k > 1) r += "." + digits.substr(1);
        int e = n - 1;
        r += e < 0 ? "e-" : "e+";
        int ae = e < 0 ? -e : e;
        if (ae < 10) r += "0";
        r += std::to_string(ae);
    }
    if (neg) out += '-';
    out += r;
}

// nlohmann dump(4): 4-space indentation, ": " after keys, "," + newline
// between members, empty containers as "{}" / "[]".
void Dump(std::string& out, const json& j, int cur)
{
    switch (j.k) {
        case json::Null: out += "null"; break;
        case json::Boolean: out += j.b ? "true" : "false"; break;
        case json::Integer: out += std::to_string(j.i); break;
        case json::Unsigned: out += std::to_string(j.u); break;
        case json::Float: DumpFloat(out, j.d); break;
        case json::String: DumpString(out, j.s); break;
        case json::Array:
            if (j.a.empty()) { out += "[]"; break; }
            out += "[\n";
            for (size_t i = 0; i < j.a.size(); i++) {
                out += std::string(cur + 4, ' ');
                Dump(out, j.a[i], cur + 4);
                out += i + 1 < j.a.size() ? ",\n" : "\n";
            }
            out += std::string(cur, ' ') + "]";
            break;
        case json::Object: {
            if (j.o.empty()) { out += "{}"; break; }
            out += "{\n";
            size_t i = 0;
            for (const auto& kv : j.o) {
                out += std::string(cur + 4, ' ');
                DumpString(out, kv.first);
                out += ": ";
                Dump(out, kv.second, cur + 4);
                out += ++i < j.o.size() ? ",\n" : "\n";
            }
            out += std::string(cur, ' ') + "}";
            break;
        }
    }
}

struct parser {
    const char* p;
    const char* end;
    std::string error;

    void ws() { while (p < end && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) p++; }
    bool fail(const char* what)
    {
        if (error.empty()) error = what;
        return false;
    }
    bool lit(const char* t)
    {
        size_t n = std::strlen(t);
        if ((size_t)(end - p) < n || std::strncmp(p, t, n) != 0) return fail("bad literal");
        p += n;
        return true;
    }
    static void utf8(std::string& s, uint32_t cp)
    {
        if (cp < 0x80) s += (char)cp;
        else if (cp < 0x800) { s += (char)(0xC0 | (cp >> 6)); s += (char)(0x80 | (cp & 63)); }
        else if (cp < 0x10000) {
            s += (char)(0xE0 | (cp >> 12)); s += (char)(0x80 | ((cp >> 6) & 63)); s += (char)(0x80 | (cp & 63));
        } else {
            s += (char)(0xF0 | (cp >> 18)); s += (char)(0x80 | ((cp >> 12) & 63));
            s += (char)(0x80 | ((cp >> 6) & 63)); s += (char)(0x80 | (cp & 63));
        }
    }
    bool hex4(uint32_t& v)
    {
        if (end - p < 4) return fail("short \\u escape");
        v = 0;
        for (int i = 0; i < 4; i++) {
            char c = *p++;
            v <<= 4;
            if (c >= '0' && c <= '9') v |= c - '0';
            else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
            else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
            else return fail("bad \\u escape");
        }
        return true;
    }
    bool str(std::string& s)
    {
        if (p >= end || *p != '"') return fail("expected string");
        p++;
        while (p < end && *p != '"') {
            char c = *p++;
            if (c != '\\') { s += c; continue; }
            if (p >= end) return fail("bad escape");
            char e = *p++;
            switch (e) {
                case '"': s += '"'; break;
                case '\\': s += '\\'; break;
                case '/': s += '/'; break;
                case 'b': s += '\b'; break;
                case 'f': s += '\f'; break;
                case 'n': s += '\n'; break;
                case 'r': s += '\r'; break;
                case 't': s += '\t'; break;
                case 'u': {
                    uint32_t v;
                    if (!hex4(v)) return false;
                    if (v >= 0xD800 && v < 0xDC00 && end - p >= 6 && p[0] == '\\' && p[1] == 'u') {
                        p += 2;
                        uint32_t lo;
                        if (!hex4(lo)) return false;
                        v = 0x10000 + ((v - 0xD800) << 10) + (lo - 0xDC00);
                    }
                    utf8(s, v);
                    break;
                }
                default: return fail("bad escape");
            }
        }
        if (p >= end) return fail("unterminated string");
        p++;
        return true;
    }
    bool value(json& j)
    {
        ws();
        if (p >= end) return fail("unexpected end");
        char c = *p;
        if (c == '{') {
            p++;
            j.k = json::Object;
            ws();
            if (p < end && *p == '}') { p++; return true; }
            for (;;) {
                ws();
                std::string key;
                if (!str(key)) return false;
                ws();
                if (p >= end || *p != ':') return fail("expected ':'");
                p++;
                if (!value(j.o[key])) return false;
                ws();
                if (p < end && *p == ',') { p++; continue; }
                if (p < end && *p == '}') { p++; return true; }
                return fail("expected ',' or '}'");
            }
        }
        if (c == '[') {
            p++;
            j.k = json::Array;
            ws();
            if (p < end && *p == ']') { p++; return true; }
            for (;;) {
                j.a.emplace_back();
                if (!value(j.a.back())) return false;
                ws();
                if (p < end && *p == ',') { p++; continue; }
                if (p < end && *p == ']') { p++; return true; }
                return fail("expected ',' or ']'");
            }
        }
        if (c == '"') { j.k = json::String; return str(j.s); }
        if (c == 't') { j = json::boolean(true); return lit("true"); }
        if (c == 'f') { j = json::boolean(false); return lit("false"); }
        if (c == 'n') { j = json(); return lit("null"); }
        // Number: integers without fraction/exponent stay integral (nlohmann's
        // number_unsigned / number_integer), everything else is a double.
        const char* q = p;
        if (q < end && *q == '-') q++;
        bool frac = false;
        while (q < end && ((*q >= '0' && *q <= '9') || *q == '.' || *q == 'e' || *q == 'E' || *q == '+' || *q == '-')) {
            if (*q == '.' || *q == 'e' || *q == 'E') frac = true;
            q++;
        }
        if (q == p) return fail("unexpected character");
        std::string t(p, q);
        p = q;
        char* e = nullptr;
        if (!frac) {
            errno = 0;
            if (t[0] == '-') {
                long long v = std::strtoll(t.c_str(), &e, 10);
                if (*e == 0 && errno == 0) { j = json::integer(v); return true; }
            } else {
                unsigned long long v = std::strtoull(t.c_str(), &e, 10);
                if (*e == 0 && errno == 0) { j = json::uinteger(v); return true; }
            }
        }
        double v = std::strtod(t.c_str(), &e);
        if (*e != 0) return fail("bad number");
        j = json::number(v);
        return true;
    }
};

// --- compressed blocks (WriteCompressed / ReadCompressed, serializer.cpp:16-44) --

bool WriteCompressed(std::ostream& Out, const void* Data, size_t Size)
{
    uLongf Bound = compressBound((uLong)Size);
    std::vector<unsigned char> Buf(std::max<size_t>(Bound, 1));
    uLongf Got = Bound;
    if (compress2(Buf.data(), &Got, static_cast<const Bytef*>(Data), (uLong)Size, Z_DEFAULT_COMPRESSION) != Z_OK)
        return false;
    if (Got > 0xFFFFFFFFul) return false;   // not representable in the reference's mz_ulong
    uint32_t N = (uint32_t)Got;
    Out.write(reinterpret_cast<const char*>(&N), sizeof N);
    Out.write(reinterpret_cast<const char*>(Buf.data()), (std::streamsize)Got);
    return (bool)Out;
}

// Accepts the 4-byte prefix (the reference's platform, and this writer) and
// an 8-byte one (mz_ulong on an LP64 build of the reference): a zlib stream
// never starts with a zero byte (CMF's low nibble is 8), while the high half
// of an 8-byte count below 4 GiB is four zero bytes.
bool ReadCompressed(std::istream& In, void* Data, size_t Size)
{
    uint32_t N = 0;
    unsigned char Next[4] = {0, 0, 0, 0};
    In.read(reinterpret_cast<char*>(&N), sizeof N);
    In.read(reinterpret_cast<char*>(Next), sizeof Next);
    if (!In) return false;
    bool Wide = Next[0] == 0 && Next[1] == 0 && Next[2] == 0 && Next[3] == 0;
    std::vector<unsigned char> Buf(std::max<size_t>(N, 4));
    size_t Have = 0;
    if (!Wide) {
        std::memcpy(Buf.data(), Next, 4);
        Have = 4;
    }
    if (N < Have) return false;
    In.read(reinterpret_cast<char*>(Buf.data() + Have), (std::streamsize)(N - Have));
    if (!In) return false;
    uLongf Got = (uLongf)Size;
    if (uncompress(static_cast<Bytef*>(Data), &Got, Buf.data(), (uLong)N) != Z_OK) return Size == 0 && N == 0;
    return Got == Size;
}

// Whether `bytes` of decompressed data can come out of what is left of the
// stream: deflate expands at most ~1032:1, so a header count beyond that is
// a corrupt file, rejected before anything is allocated from it.
bool PlausibleInflated(std::istream& In, uint64_t bytes)
{
    std::streampos At = In.tellg();
    if (At < 0) return false;
    In.seekg(0, std::ios::end);
    std::streampos End = In.tellg();
    In.seekg(At);
    if (End < At || !In) return false;
    uint64_t Left = (uint64_t)(End - At);
    return bytes <= 1100 * Left + 4096;
}

constexpr uint32_t MAGIC_TEXTURE = 0x54455820u;   // 'TEX '
constexpr uint32_t MAGIC_MESH = 0x4D455348u;      // 'MESH'
constexpr uint32_t MAGIC_SPECTRUM = 0x53504543u;  // 'SPEC'

static_assert(sizeof(mesh_face) == 12, "mesh_face layout (scene.hpp:198-201)");
static_assert(sizeof(mesh_node) == 36, "mesh_node layout (scene.hpp:210-216)");
static_assert(sizeof(mesh_vertex) == 32, "mesh_vertex layout (scene.hpp:203-208)");
static_assert(sizeof(vec4) == 16, "texture pixel layout");

std::string MakeFileName(const std::string& Name, const char* Extension)
{
    std::string Str = Name;
    for (char& Ch : Str)
        if (!std::isalnum(static_cast<unsigned char>(Ch))) Ch = '_';
    size_t first = 0;
    while (first < Str.size() && std::isspace(static_cast<unsigned char>(Str[first]))) first++;
    Str.erase(0, first);
    return Str + "." + Extension;
}

// --- field helpers -------------------------------------------------------------

json V2(vec2 v) { json j; j.push_back(json::number(v.x)); j.push_back(json::number(v.y)); return j; }
json V3(vec3 v)
{
    json j;
    j.push_back(json::number(v.x)); j.push_back(json::number(v.y)); j.push_back(json::number(v.z));
    return j;
}
json F(float v) { return json::number(v); }
json U(uint32_t v) { return json::uinteger(v); }
json I(int64_t v) { return json::integer(v); }

void Get(const json& J, const char* Key, float& Out)
{
    const json* v = J.find(Key);
    if (v && v->is_number()) Out = (float)v->num();
}
void Get(const json& J, const char* Key, uint32_t& Out)
{
    const json* v = J.find(Key);
    if (v && v->is_number()) Out = (uint32_t)v->inum();
}
void Get(const json& J, const char* Key, int& Out)
{
    const json* v = J.find(Key);
    if (v && v->is_number()) Out = (int)v->inum();
}
void Get(const json& J, const char* Key, bool& Out)
{
    const json* v = J.find(Key);
    if (v && v->k == json::Boolean) Out = v->b;
}
void Get(const json& J, const char* Key, std::string& Out)
{
    const json* v = J.find(Key);
    if (v && v->k == json::String) Out = v->s;
}
template <int N>
void GetVec(const json& J, const char* Key, float* Out)
{
    const json* v = J.find(Key);
    if (!v || v->k != json::Array || v->a.size() < N) return;
    for (int i = 0; i < N; i++) Out[i] = (float)v->a[i].num();
}
void Get(const json& J, const char* Key, vec2& Out) { GetVec<2>(J, Key, &Out.x); }
void Get(const json& J, const char* Key, vec3& Out) { GetVec<3>(J, Key, &Out.x); }

struct serializer {
    std::filesystem::path SceneFilePath;
    std::filesystem::path DirectoryPath;
    std::unordered_map<const texture*, int> TextureIndex;
    std::unordered_map<const material*, int> MaterialIndex;
    std::unordered_map<const mesh*, int> MeshIndex;
    scene* Scene = nullptr;
    std::string Error;
    std::unordered_map<std::string, int> UsedFileNames;

    // MakeFileName, numbered on a collision (extension, see the header).
    std::string UniqueFileName(json& J, const std::string& Name, const char* Extension)
    {
        std::string File = MakeFileName(Name, Extension);
        int& Uses = UsedFileNames[File];
        if (Uses++ == 0) return File;
        for (int n = Uses + 1;; n++) {
            std::string Alt = MakeFileName(Name + "_" + std::to_string(n), Extension);
            if (UsedFileNames[Alt]++ == 0) {
                J["FileName"] = json::string(Alt);
                return Alt;
            }
        }
    }

    static std::string StoredFileName(const json& J, const std::string& Name, const char* Extension)
    {
        const json* F = J.find("FileName");
        return F && F->k == json::String ? F->s : MakeFileName(Name, Extension);
    }

    json Ref(const texture* T) { auto it = TextureIndex.find(T); return I(it == TextureIndex.end() ? -1 : it->second); }
    json Ref(const material* M) { auto it = MaterialIndex.find(M); return I(it == MaterialIndex.end() ? -1 : it->second); }
    json Ref(const mesh* M) { auto it = MeshIndex.find(M); return I(it == MeshIndex.end() ? -1 : it->second); }

    template <class T>
    T* Deref(const json& J, const char* Key, const std::vector<T*>& Pool, T* Default)
    {
        const json* v = J.find(Key);
        if (!v || !v->is_number()) return Default;
        int64_t i = v->inum();
        return (i >= 0 && i < (int64_t)Pool.size()) ? Pool[(size_t)i] : nullptr;
    }

    // --- writing ---

    bool WriteTexture(json& J, const texture& T)
    {
        J["Type"] = U(T.Type);
        J["Name"] = json::string(T.Name);
        J["EnableNearestFiltering"] = json::boolean(T.EnableNearestFiltering);
        std::ofstream File(DirectoryPath / UniqueFileName(J, T.Name, "texture"), std::ios::binary);
        uint32_t Header[4] = {MAGIC_TEXTURE, 0, T.Width, T.Height};
        File.write(reinterpret_cast<const char*>(Header), sizeof Header);
        size_t n = (size_t)T.Width * T.Height;
        if (T.Pixels.size() < n) { Error = "texture '" + T.Name + "' has fewer pixels than Width*Height"; return false; }
        if (!WriteCompressed(File, T.Pixels.data(), sizeof(vec4) * n)) { Error = "cannot write texture " + T.Name; return false; }
        return true;
    }

    void WriteMaterial(json& J, const material& M)
    {
        J["Type"] = U(M.Type);
        J["Name"] = json::string(M.Name);
        J["Flags"] = U(M.Flags);
        J["Opacity"] = F(M.Opacity);
        switch (M.Type) {
            case PT_MATERIAL_TYPE_BASIC_DIFFUSE:        // basic_diffuse.hpp:44-51
                J["BaseColor"] = V3(M.BaseColor);
                J["BaseTexture"] = Ref(M.BaseTexture);
                break;
            case PT_MATERIAL_TYPE_BASIC_METAL:          // basic_metal.hpp:74-87
                J["BaseColor"] = V3(M.BaseColor);
                J["BaseTexture"] = Ref(M.BaseTexture);
                J["SpecularColor"] = V3(M.SpecularColor);
                J["SpecularTexture"] = Ref(M.SpecularTexture);
                J["Roughness"] = F(M.Roughness);
                J["RoughnessTexture"] = Ref(M.RoughnessTexture);
                J["RoughnessAnisotropy"] = F(M.RoughnessAnisotropy);
                J["RoughnessAnisotropyTexture"] = Ref(M.RoughnessAnisotropyTexture);
                break;
            case PT_MATERIAL_TYPE_BASIC_TRANSLUCENT:    // basic_translucent.hpp:87-103
                J["IOR"] = F(M.IOR);
                J["AbbeNumber"] = F(M.AbbeNumber);
                J["Roughness"] = F(M.Roughness);
                J["RoughnessTexture"] = Ref(M.RoughnessTexture);
                J["RoughnessAnisotropy"] = F(M.RoughnessAnisotropy);
                J["RoughnessAnisotropyTexture"] = Ref(M.RoughnessAnisotropyTexture);
                J["TransmissionColor"] = V3(M.TransmissionColor);
                J["TransmissionDepth"] = F(M.TransmissionDepth);
                J["ScatteringColor"] = V3(M.ScatteringColor);
                J["ScatteringAnisotropy"] = F(M.ScatteringAnisotropy);
                break;
            case PT_MATERIAL_TYPE_OPENPBR:              // openpbr.hpp:183-217
                J["BaseWeight"] = F(M.BaseWeight);
                J["BaseColor"] = V3(M.BaseColor);
                J["BaseColorTexture"] = Ref(M.BaseTexture);
                J["BaseMetalness"] = F(M.BaseMetalness);
                J["BaseDiffuseRoughness"] = F(M.BaseDiffuseRoughness);
                J["SpecularWeight"] = F(M.SpecularWeight);
                J["SpecularColor"] = V3(M.SpecularColor);
                J["SpecularRoughness"] = F(M.Roughness);
                J["SpecularRoughnessTexture"] = Ref(M.RoughnessTexture);
                J["SpecularRoughnessAnisotropy"] = F(M.RoughnessAnisotropy);
                J["SpecularIOR"] = F(M.SpecularIOR);
                J["TransmissionWeight"] = F(M.TransmissionWeight);
                J["TransmissionColor"] = V3(M.TransmissionColor);
                J["TransmissionDepth"] = F(M.TransmissionDepth);
                J["TransmissionScatter"] = V3(M.TransmissionScatter);
                J["TransmissionScatterAnisotropy"] = F(M.TransmissionScatterAnisotropy);
                J["TransmissionDispersionScale"] = F(M.TransmissionDispersionScale);
                J["TransmissionDispersionAbbeNumber"] = F(M.TransmissionDispersionAbbeNumber);
                J["CoatWeight"] = F(M.CoatWeight);
                J["CoatColor"] = V3(M.CoatColor);
                J["CoatRoughness"] = F(M.CoatRoughness);
                J["CoatRoughnessAnisotropy"] = F(M.CoatRoughnessAnisotropy);
                J["CoatIOR"] = F(M.CoatIOR);
                J["CoatDarkening"] = F(M.CoatDarkening);
                J["EmissionLuminance"] = F(M.EmissionLuminance);
                J["EmissionColor"] = V3(M.EmissionColor);
                J["EmissionColorTexture"] = Ref(M.EmissionColorTexture);
                J["LayerBounceLimit"] = I(M.LayerBounceLimit);
                break;
            default: break;
        }
    }

    bool WriteMesh(json& J, const mesh& M)
    {
        J["Name"] = json::string(M.Name);
        std::ofstream File(DirectoryPath / UniqueFileName(J, M.Name, "mesh"), std::ios::binary);
        uint32_t Header[4] = {MAGIC_MESH, 0, (uint32_t)M.Faces.size(), (uint32_t)M.Nodes.size()};
        File.write(reinterpret_cast<const char*>(Header), sizeof Header);
        bool ok = WriteCompressed(File, M.Faces.data(), sizeof(mesh_face) * M.Faces.size()) &&
                  WriteCompressed(File, M.Nodes.data(), sizeof(mesh_node) * M.Nodes.size());
        // Extension block (see the header comment): the vertices.
        uint64_t VertexCount = M.Vertices.size();
        File.write(reinterpret_cast<const char*>(&VertexCount), sizeof VertexCount);
        ok = ok && WriteCompressed(File, M.Vertices.data(), sizeof(mesh_vertex) * M.Vertices.size());
        if (!ok || !File) { Error = "cannot write mesh " + M.Name; return false; }
        return true;
    }

    void WriteEntity(json& J, const entity& E)
    {
        J["Type"] = I(E.Type);
        J["Position"] = V3(E.Transform.Position);
        J["Rotation"] = V3(E.Transform.Rotation);
        J["Scale"] = V3(E.Transform.Scale);
        J["Name"] = json::string(E.Name);
        J["Active"] = json::boolean(E.Active);
        J["Material"] = Ref(E.Material);
        switch (E.Type) {
            case ENTITY_TYPE_ROOT:
                J["ScatterRate"] = F(E.ScatterRate);
                J["SkyboxBrightness"] = F(E.SkyboxBrightness);
                J["SkyboxTexture"] = Ref(E.SkyboxTexture);
                J["SkyboxSamplingProbability"] = F(E.SkyboxSamplingProbability);   // extension
                break;
            case ENTITY_TYPE_CAMERA:
                J["CameraModel"] = U(E.CameraModel);
                J["Pinhole"]["FieldOfViewInDegrees"] = F(E.PinholeFieldOfViewInDegrees);
                J["Pinhole"]["ApertureDiameterInMM"] = F(E.PinholeApertureDiameterInMM);
                J["ThinLens"]["SensorSizeInMM"] = V2(E.ThinLensSensorSizeInMM);
                J["ThinLens"]["FocalLengthInMM"] = F(E.ThinLensFocalLengthInMM);
                J["ThinLens"]["ApertureDiameterInMM"] = F(E.ThinLensApertureDiameterInMM);
                J["ThinLens"]["FocusDistance"] = F(E.ThinLensFocusDistance);
                break;
            case ENTITY_TYPE_MESH_INSTANCE:
                J["Mesh"] = Ref(E.Mesh);
                break;
            default: break;
        }
        json& Children = J["Children"];   // null when there are none, like nlohmann
        for (const entity* C : E.Children) WriteEntity(Children.push_back(json()), *C);
    }

    // --- reading ---

    bool ReadTexture(const json& J, texture& T)
    {
        Get(J, "Type", T.Type);
        Get(J, "Name", T.Name);
        Get(J, "EnableNearestFiltering", T.EnableNearestFiltering);
        std::ifstream File(DirectoryPath / StoredFileName(J, T.Name, "texture"), std::ios::binary);
        uint32_t Header[4] = {0, 0, 0, 0};
        File.read(reinterpret_cast<char*>(Header), sizeof Header);
        if (!File || Header[0] != MAGIC_TEXTURE) { Error = "bad texture file for '" + T.Name + "'"; return false; }
        T.Width = Header[2];
        T.Height = Header[3];
        if (!PlausibleInflated(File, (uint64_t)T.Width * T.Height * sizeof(vec4))) {
            Error = "corrupt texture data for '" + T.Name + "'";
            return false;
        }
        T.Pixels.resize((size_t)T.Width * T.Height);
        if (!ReadCompressed(File, T.Pixels.data(), sizeof(vec4) * T.Pixels.size())) {
            Error = "corrupt texture data for '" + T.Name + "'";
            return false;
        }
        return true;
    }

    void ReadMaterial(const json& J, material& M)
    {
        const auto& Tx = Scene->Textures;
        Get(J, "Name", M.Name);
        Get(J, "Flags", M.Flags);
        Get(J, "Opacity", M.Opacity);
        switch (M.Type) {
            case PT_MATERIAL_TYPE_BASIC_DIFFUSE:
                Get(J, "BaseColor", M.BaseColor);
                M.BaseTexture = Deref(J, "BaseTexture", Tx, M.BaseTexture);
                break;
            case PT_MATERIAL_TYPE_BASIC_METAL:
                Get(J, "BaseColor", M.BaseColor);
                M.BaseTexture = Deref(J, "BaseTexture", Tx, M.BaseTexture);
                Get(J, "SpecularColor", M.SpecularColor);
                M.SpecularTexture = Deref(J, "SpecularTexture", Tx, M.SpecularTexture);
                Get(J, "Roughness", M.Roughness);
                M.RoughnessTexture = Deref(J, "RoughnessTexture", Tx, M.RoughnessTexture);
                Get(J, "RoughnessAnisotropy", M.RoughnessAnisotropy);
                M.RoughnessAnisotropyTexture = Deref(J, "RoughnessAnisotropyTexture", Tx, M.RoughnessAnisotropyTexture);
                break;
            case PT_MATERIAL_TYPE_BASIC_TRANSLUCENT:
                Get(J, "IOR", M.IOR);
                Get(J, "AbbeNumber", M.AbbeNumber);
                Get(J, "Roughness", M.Roughness);
                M.RoughnessTexture = Deref(J, "RoughnessTexture", Tx, M.RoughnessTexture);
                Get(J, "RoughnessAnisotropy", M.RoughnessAnisotropy);
                M.RoughnessAnisotropyTexture = Deref(J, "RoughnessAnisotropyTexture", Tx, M.RoughnessAnisotropyTexture);
                Get(J, "TransmissionColor", M.TransmissionColor);
                Get(J, "TransmissionDepth", M.TransmissionDepth);
                Get(J, "ScatteringColor", M.ScatteringColor);
                Get(J, "ScatteringAnisotropy", M.ScatteringAnisotropy);
                break;
            case PT_MATERIAL_TYPE_OPENPBR:
                Get(J, "BaseWeight", M.BaseWeight);
                Get(J, "BaseColor", M.BaseColor);
                M.BaseTexture = Deref(J, "BaseColorTexture", Tx, M.BaseTexture);
                Get(J, "BaseMetalness", M.BaseMetalness);
                Get(J, "BaseDiffuseRoughness", M.BaseDiffuseRoughness);
                Get(J, "SpecularWeight", M.SpecularWeight);
                Get(J, "SpecularColor", M.SpecularColor);
                Get(J, "SpecularRoughness", M.Roughness);
                M.RoughnessTexture = Deref(J, "SpecularRoughnessTexture", Tx, M.RoughnessTexture);
                Get(J, "SpecularRoughnessAnisotropy", M.RoughnessAnisotropy);
                Get(J, "SpecularIOR", M.SpecularIOR);
                Get(J, "TransmissionWeight", M.TransmissionWeight);
                Get(J, "TransmissionColor", M.TransmissionColor);
                Get(J, "TransmissionDepth", M.TransmissionDepth);
                Get(J, "TransmissionScatter", M.TransmissionScatter);
                Get(J, "TransmissionScatterAnisotropy", M.TransmissionScatterAnisotropy);
                Get(J, "TransmissionDispersionScale", M.TransmissionDispersionScale);
                Get(J, "TransmissionDispersionAbbeNumber", M.TransmissionDispersionAbbeNumber);
                Get(J, "CoatWeight", M.CoatWeight);
                Get(J, "CoatColor", M.CoatColor);
                Get(J, "CoatRoughness", M.CoatRoughness);
                Get(J, "CoatRoughnessAnisotropy", M.CoatRoughnessAnisotropy);
                Get(J, "CoatIOR", M.CoatIOR);
                Get(J, "CoatDarkening", M.CoatDarkening);
                Get(J, "EmissionLuminance", M.EmissionLuminance);
                Get(J, "EmissionColor", M.EmissionColor);
                M.EmissionColorTexture = Deref(J, "EmissionColorTexture", Tx, M.EmissionColorTexture);
                Get(J, "LayerBounceLimit", M.LayerBounceLimit);
                break;
            default: break;
        }
    }

    static uint32_t NodeDepth(const mesh& M, uint32_t Index, uint32_t Level)
    {
        if (Index >= M.Nodes.size() || Level > 64) return Level;
        const mesh_node& N = M.Nodes[Index];
        if (N.FaceEndIndex > 0 || N.ChildNodeIndex == 0) return Level;
        return std::max(NodeDepth(M, N.ChildNodeIndex, Level + 1), NodeDepth(M, N.ChildNodeIndex + 1, Level + 1));
    }

    bool ReadMesh(const json& J, mesh& M)
    {
        Get(J, "Name", M.Name);
        std::ifstream File(DirectoryPath / StoredFileName(J, M.Name, "mesh"), std::ios::binary);
        uint32_t Header[4] = {0, 0, 0, 0};
        File.read(reinterpret_cast<char*>(Header), sizeof Header);
        if (!File || Header[0] != MAGIC_MESH) { Error = "bad mesh file for '" + M.Name + "'"; return false; }
        if (!PlausibleInflated(File, (uint64_t)Header[2] * sizeof(mesh_face) + (uint64_t)Header[3] * sizeof(mesh_node))) {
            Error = "corrupt mesh data for '" + M.Name + "'";
            return false;
        }
        M.Faces.resize(Header[2]);
        M.Nodes.resize(Header[3]);
        if (!ReadCompressed(File, M.Faces.data(), sizeof(mesh_face) * M.Faces.size()) ||
            !ReadCompressed(File, M.Nodes.data(), sizeof(mesh_node) * M.Nodes.size())) {
            Error = "corrupt mesh data for '" + M.Name + "'";
            return false;
        }
        uint64_t VertexCount = 0;
        File.read(reinterpret_cast<char*>(&VertexCount), sizeof VertexCount);
        if (File && VertexCount < (1ull << 32) && !PlausibleInflated(File, VertexCount * sizeof(mesh_vertex))) {
            Error = "corrupt vertex data for '" + M.Name + "'";
            return false;
        }
        if (File && VertexCount < (1ull << 32)) {
            M.Vertices.resize((size_t)VertexCount);
            if (!ReadCompressed(File, M.Vertices.data(), sizeof(mesh_vertex) * M.Vertices.size())) {
                Error = "corrupt vertex data for '" + M.Name + "'";
                return false;
            }
        } else {
            M.Vertices.clear();   // a reference-written file: no vertices
        }
        M.Depth = M.Nodes.empty() ? 0 : NodeDepth(M, 0, 0);
        return true;
    }

    void ReadEntity(const json& J, entity& E, std::vector<entity*>& Owner)
    {
        Get(J, "Position", E.Transform.Position);
        Get(J, "Rotation", E.Transform.Rotation);
        Get(J, "Scale", E.Transform.Scale);
        Get(J, "Name", E.Name);
        Get(J, "Active", E.Active);
        E.Material = Deref(J, "Material", Scene->Materials, E.Material);
        switch (E.Type) {
            case ENTITY_TYPE_ROOT:
                Get(J, "ScatterRate", E.ScatterRate);
                Get(J, "SkyboxBrightness", E.SkyboxBrightness);
                E.SkyboxTexture = Deref(J, "SkyboxTexture", Scene->Textures, E.SkyboxTexture);
                Get(J, "SkyboxSamplingProbability", E.SkyboxSamplingProbability);
                break;
            case ENTITY_TYPE_CAMERA: {
                Get(J, "CameraModel", E.CameraModel);
                static const json None;
                const json* P = J.find("Pinhole");
                const json* T = J.find("ThinLens");
                Get(P ? *P : None, "FieldOfViewInDegrees", E.PinholeFieldOfViewInDegrees);
                Get(P ? *P : None, "ApertureDiameterInMM", E.PinholeApertureDiameterInMM);
                Get(T ? *T : None, "SensorSizeInMM", E.ThinLensSensorSizeInMM);
                Get(T ? *T : None, "FocalLengthInMM", E.ThinLensFocalLengthInMM);
                Get(T ? *T : None, "ApertureDiameterInMM", E.ThinLensApertureDiameterInMM);
                Get(T ? *T : None, "FocusDistance", E.ThinLensFocusDistance);
                break;
            }
            case ENTITY_TYPE_MESH_INSTANCE:
                E.Mesh = Deref(J, "Mesh", Scene->Meshes, E.Mesh);
                break;
            default: break;
        }
        const json* Children = J.find("Children");
        if (!Children || Children->k != json::Array) return;
        for (const json& CJ : Children->a) {
            entity* C = new entity;
            Owner.push_back(C);
            int Type = 0;
            Get(CJ, "Type", Type);
            C->Type = static_cast<entity_type>(Type);
            C->Parent = &E;
            E.Children.push_back(C);
            ReadEntity(CJ, *C, Owner);
        }
    }
};

}  // namespace

bool SaveScene(const char* Path, scene* Scene, std::string* Error)
{
    serializer S;
    S.SceneFilePath = Path;
    S.DirectoryPath = S.SceneFilePath.parent_path();
    if (S.DirectoryPath.empty()) S.DirectoryPath = ".";
    S.Scene = Scene;
    std::error_code ec;
    std::filesystem::create_directory(S.DirectoryPath, ec);

    json J;
    for (size_t i = 0; i < Scene->Textures.size(); i++) S.TextureIndex[Scene->Textures[i]] = (int)i;
    for (size_t i = 0; i < Scene->Materials.size(); i++) S.MaterialIndex[Scene->Materials[i]] = (int)i;
    for (size_t i = 0; i < Scene->Meshes.size(); i++) S.MeshIndex[Scene->Meshes[i]] = (int)i;
    bool ok = true;
    for (const texture* T : Scene->Textures) ok = ok && S.WriteTexture(J["Textures"].push_back(json()), *T);
    for (const material* M : Scene->Materials) S.WriteMaterial(J["Materials"].push_back(json()), *M);
    for (const mesh* M : Scene->Meshes) ok = ok && S.WriteMesh(J["Meshes"].push_back(json()), *M);
    for (const prefab* P : Scene->Prefabs)
        if (P->Entity) S.WriteEntity(J["Prefabs"].push_back(json()), *P->Entity);
    S.WriteEntity(J["Root"], Scene->Root);
    if (ok) {
        std::string Text;
        Dump(Text, J, 0);
        std::ofstream File(S.SceneFilePath);
        File << Text;
        if (!File) { S.Error = "cannot write " + S.SceneFilePath.string(); ok = false; }
    }
    // The RGB -> spectrum coefficient table (serializer.cpp:481-509).
    if (ok) {
        parametric_spectrum_table* Table = Scene->RGBSpectrumTable ? Scene->RGBSpectrumTable : GetSharedSpectrumTable();
        BuildParametricSpectrumTableForSRGB(Table, 0);   // only chains not yet evaluated
        std::ofstream File(S.DirectoryPath / "spectrum.dat", std::ios::binary);
        uint32_t Header[2] = {MAGIC_SPECTRUM, 0};
        File.write(reinterpret_cast<const char*>(Header), sizeof Header);
        if (!WriteCompressed(File, Table->Coefficients, sizeof(Table->Coefficients))) {
            S.Error = "cannot write spectrum.dat";
            ok = false;
        }
    }
    if (!ok && Error) *Error = S.Error;
    return ok;
}

scene* LoadScene(const char* Path, std::string* Error)
{
    serializer S;
    S.SceneFilePath = Path;
    S.DirectoryPath = S.SceneFilePath.parent_path();
    if (S.DirectoryPath.empty()) S.DirectoryPath = ".";
    auto Fail = [&](const std::string& Message, scene* Scene) -> scene* {
        if (Error) *Error = Message;
        delete Scene;
        return nullptr;
    };
    std::ifstream In(S.SceneFilePath, std::ios::binary);
    if (!In) return Fail(std::string("cannot open ") + Path, nullptr);
    std::stringstream Buf;
    Buf << In.rdbuf();
    std::string Text = Buf.str();
    json J;
    parser Ps{Text.data(), Text.data() + Text.size(), {}};
    if (!Ps.value(J)) return Fail("scene JSON: " + Ps.error, nullptr);

    scene* Scene = CreateEmptyScene();
    S.Scene = Scene;
    static const json None;
    const json* Tx = J.find("Textures");
    const json* Mt = J.find("Materials");
    const json* Ms = J.find("Meshes");
    const json* Pf = J.find("Prefabs");
    // Objects are created first so that references by index resolve
    // (serializer.cpp:402-426).
    for (size_t i = 0; Tx && i < Tx->a.size(); i++) Scene->Textures.push_back(new texture);
    for (size_t i = 0; Mt && i < Mt->a.size(); i++) {
        uint32_t Type = PT_MATERIAL_TYPE_BASIC_DIFFUSE;
        Get(Mt->a[i], "Type", Type);
        CreateMaterial(Scene, Type, "");
    }
    for (size_t i = 0; Ms && i < Ms->a.size(); i++) Scene->Meshes.push_back(new mesh);
    for (size_t i = 0; Tx && i < Tx->a.size(); i++)
        if (!S.ReadTexture(Tx->a[i], *Scene->Textures[i])) return Fail(S.Error, Scene);
    for (size_t i = 0; Mt && i < Mt->a.size(); i++) S.ReadMaterial(Mt->a[i], *Scene->Materials[i]);
    for (size_t i = 0; Ms && i < Ms->a.size(); i++)
        if (!S.ReadMesh(Ms->a[i], *Scene->Meshes[i])) return Fail(S.Error, Scene);
    for (size_t i = 0; Pf && i < Pf->a.size(); i++) {
        prefab* P = new prefab;
        Scene->Prefabs.push_back(P);
        P->Entity = new entity;
        P->Owned.push_back(P->Entity);
        int Type = 0;
        Get(Pf->a[i], "Type", Type);
        P->Entity->Type = static_cast<entity_type>(Type);
        S.ReadEntity(Pf->a[i], *P->Entity, P->Owned);
    }
    const json* Root = J.find("Root");
    S.ReadEntity(Root ? *Root : None, Scene->Root, Scene->Entities);

    std::ifstream Spec(S.DirectoryPath / "spectrum.dat", std::ios::binary);
    if (Spec) {
        uint32_t Header[2] = {0, 0};
        Spec.read(reinterpret_cast<char*>(Header), sizeof Header);
        if (!Spec || Header[0] != MAGIC_SPECTRUM) return Fail("bad spectrum.dat", Scene);
        auto* Table = new parametric_spectrum_table;
        if (!ReadCompressed(Spec, Table->Coefficients, sizeof(Table->Coefficients))) {
            delete Table;
            return Fail("corrupt spectrum.dat", Scene);
        }
        for (int i = 0; i < parametric_spectrum_table::CHAIN_COUNT; i++) Table->ChainReady[i].store(1);
        Scene->RGBSpectrumTable = Table;
        Scene->OwnsSpectrumTable = true;
    }
    Scene->DirtyFlags = PT_SCENE_DIRTY_ALL;
    return Scene;
}

}  // namespace pth
