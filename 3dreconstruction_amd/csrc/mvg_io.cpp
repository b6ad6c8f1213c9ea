// Stage-boundary file formats of the reference's file-staged sparseBuilder
// flow, read and written natively so the GPU matcher
// drops into matchPair() / match() (src/sparseBuilder/sparseBuilder.cpp:758-1023)
// without OpenMVG.  OpenMVG is un-vendored in the reference tree and absent
// here, so every layout below is a restatement of its published code at the
// call sites the reference uses (parity unpinned):
//
//   sfm_data.json        cereal JSON of SfM_Data; only VIEWS are read
//                        (Load(..., ESfM_Data(VIEWS|INTRINSICS)) :773, :835)
//   image_describer.json cereal JSON; "regions_type" must be SIFT_Regions
//                        (Init_region_type_from_file :851)
//   <stem>.desc          saveDescsToBinFile: uint64 count, count x 128 uint8
//   <stem>.feat          saveFeatsToFile (SIOPointFeature): "x y scale orient\n"
//   pairs.bin            savePairs / loadPairs: text, "I J1 J2 ...\n" per line
//                        (:801, :948) — a text file despite its name
//   matches.putative.bin Save(PairWiseMatches) with cereal PortableBinary:
//                        uint8 1 (little endian), uint64 #pairs, then per pair
//                        uint32 I, uint32 J, uint64 n, n x (uint32 i, uint32 j)
//                        (:986); ".txt" gives "I J\nn\ni j\n..." instead
//   preemptive_pairs.txt savePairs(getPairs(matches)) (:995-1001)
#include <sys/stat.h>

#include <algorithm>
#include <array>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <set>
#include <sstream>
#include <string>
#include <utility>
#include <vector>

#include "common.h"

namespace sfm {
namespace {

// ---------------------------------------------------------------------------
// minimal JSON reader (cereal's JSONOutputArchive output)
// ---------------------------------------------------------------------------
struct Json {
    enum Kind { Null, Bool, Num, Str, Arr, Obj } kind = Null;
    double num = 0.0;
    bool b = false;
    std::string str;
    std::vector<Json> arr;
    std::vector<std::pair<std::string, Json>> obj;   // insertion order kept

    const Json* get(const char* k) const {
        if (kind != Obj) return nullptr;
        for (const auto& kv : obj)
            if (kv.first == k) return &kv.second;
        return nullptr;
    }
};

class JsonParser {
   public:
    explicit JsonParser(const std::string& s) : s_(s) {}
    Json parse() {
        Json v = value();
        ws();
        SFM_REQUIRE(i_ == s_.size(), SFM_ERR_INVALID_ARG, "json: trailing data at offset %zu", i_);
        return v;
    }

   private:
    const std::string& s_;
    size_t i_ = 0;

    void ws() {
        while (i_ < s_.size() && (s_[i_] == ' ' || s_[i_] == '\n' || s_[i_] == '\r' || s_[i_] == '\t')) ++i_;
    }
    char peek() {
        ws();
        SFM_REQUIRE(i_ < s_.size(), SFM_ERR_INVALID_ARG, "json: unexpected end");
        return s_[i_];
    }
    void expect(char c) {
        SFM_REQUIRE(peek() == c, SFM_ERR_INVALID_ARG, "json: expected '%c' at offset %zu", c, i_);
        ++i_;
    }
    bool lit(const char* w) {
        const size_t n = std::strlen(w);
        if (s_.compare(i_, n, w) == 0) {
            i_ += n;
            return true;
        }
        return false;
    }
    static void utf8(std::string& out, unsigned cp) {
        if (cp < 0x80) {
            out += (char)cp;
        } else if (cp < 0x800) {
            out += (char)(0xC0 | (cp >> 6));
            out += (char)(0x80 | (cp & 0x3F));
        } else if (cp < 0x10000) {
            out += (char)(0xE0 | (cp >> 12));
            out += (char)(0x80 | ((cp >> 6) & 0x3F));
            out += (char)(0x80 | (cp & 0x3F));
        } else {
            out += (char)(0xF0 | (cp >> 18));
            out += (char)(0x80 | ((cp >> 12) & 0x3F));
            out += (char)(0x80 | ((cp >> 6) & 0x3F));
            out += (char)(0x80 | (cp & 0x3F));
        }
    }
    unsigned hex4() {
        SFM_REQUIRE(i_ + 4 <= s_.size(), SFM_ERR_INVALID_ARG, "json: short \\u escape");
        unsigned v = 0;
        for (int k = 0; k < 4; ++k) {
            const char c = s_[i_++];
            v <<= 4;
            if (c >= '0' && c <= '9') v |= (unsigned)(c - '0');
            else if (c >= 'a' && c <= 'f') v |= (unsigned)(c - 'a' + 10);
            else if (c >= 'A' && c <= 'F') v |= (unsigned)(c - 'A' + 10);
            else SFM_REQUIRE(false, SFM_ERR_INVALID_ARG, "json: bad \\u escape");
        }
        return v;
    }
    std::string string() {
        expect('"');
        std::string out;
        while (true) {
            SFM_REQUIRE(i_ < s_.size(), SFM_ERR_INVALID_ARG, "json: unterminated string");
            const char c = s_[i_++];
            if (c == '"') break;
            if (c != '\\') {
                out += c;
                continue;
            }
            SFM_REQUIRE(i_ < s_.size(), SFM_ERR_INVALID_ARG, "json: unterminated escape");
            const char e = s_[i_++];
            switch (e) {
                case '"': out += '"'; break;
                case '\\': out += '\\'; break;
                case '/': out += '/'; break;
                case 'b': out += '\b'; break;
                case 'f': out += '\f'; break;
                case 'n': out += '\n'; break;
                case 'r': out += '\r'; break;
                case 't': out += '\t'; break;
                case 'u': {
                    unsigned cp = hex4();
                    if (cp >= 0xD800 && cp < 0xDC00 && i_ + 6 <= s_.size() && s_[i_] == '\\' && s_[i_ + 1] == 'u') {
                        i_ += 2;
                        const unsigned lo = hex4();
                        cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
                    }
                    utf8(out, cp);
                    break;
                }
                default: SFM_REQUIRE(false, SFM_ERR_INVALID_ARG, "json: bad escape '\\%c'", e);
            }
        }
        return out;
    }
    Json value() {
        Json v;
        const char c = peek();
        if (c == '{') {
            ++i_;
            v.kind = Json::Obj;
            if (peek() == '}') {
                ++i_;
                return v;
            }
            while (true) {
                std::string k = string();
                expect(':');
                v.obj.emplace_back(std::move(k), value());
                if (peek() == ',') {
                    ++i_;
                    continue;
                }
                expect('}');
                return v;
            }
        }
        if (c == '[') {
            ++i_;
            v.kind = Json::Arr;
            if (peek() == ']') {
                ++i_;
                return v;
            }
            while (true) {
                v.arr.push_back(value());
                if (peek() == ',') {
                    ++i_;
                    continue;
                }
                expect(']');
                return v;
            }
        }
        if (c == '"') {
            v.kind = Json::Str;
            v.str = string();
            return v;
        }
        if (lit("true")) { v.kind = Json::Bool; v.b = true; return v; }
        if (lit("false")) { v.kind = Json::Bool; return v; }
        if (lit("null")) return v;
        const char* b = s_.c_str() + i_;
        char* e = nullptr;
        v.num = std::strtod(b, &e);
        SFM_REQUIRE(e != b, SFM_ERR_INVALID_ARG, "json: bad value at offset %zu", i_);
        v.kind = Json::Num;
        i_ += (size_t)(e - b);
        return v;
    }
};

std::string slurp(const char* path) {
    std::ifstream f(path, std::ios::binary);
    SFM_REQUIRE(f.good(), SFM_ERR_INVALID_ARG, "cannot open %s", path);
    std::ostringstream ss;
    ss << f.rdbuf();
    return ss.str();
}

bool is_file(const std::string& p) {
    struct stat st;
    return ::stat(p.c_str(), &st) == 0 && S_ISREG(st.st_mode);
}

// stlplus::create_filespec(dir, name)
std::string filespec(const std::string& dir, const std::string& name) {
    if (dir.empty()) return name;
    if (dir.back() == '/') return dir + name;
    return dir + "/" + name;
}

// stlplus::basename_part: file name without directory and last extension
std::string basename_part(const std::string& p) {
    const size_t s = p.find_last_of('/');
    std::string f = s == std::string::npos ? p : p.substr(s + 1);
    const size_t d = f.find_last_of('.');
    if (d != std::string::npos && d > 0) f = f.substr(0, d);
    return f;
}

uint32_t as_u32(const Json* v, const char* what) {
    SFM_REQUIRE(v && v->kind == Json::Num && v->num >= 0 && v->num <= 4294967295.0 && std::floor(v->num) == v->num,
                SFM_ERR_INVALID_ARG, "sfm_data: bad or missing %s", what);
    return (uint32_t)v->num;
}

// The object holding a view's fields: cereal writes a polymorphic
// shared_ptr<View> as {"polymorphic_id", ["polymorphic_name",] "ptr_wrapper":
// {"id", "data": {...}}}; a derived ViewPriors nests the base fields.
const Json* view_fields(const Json& v) {
    if (v.kind != Json::Obj) return nullptr;
    if (v.get("filename") && v.get("id_view")) return &v;
    for (const auto& kv : v.obj) {
        const Json* r = view_fields(kv.second);
        if (r) return r;
    }
    return nullptr;
}

struct View {
    uint32_t id_view = 0, id_intrinsic = 0, id_pose = 0, width = 0, height = 0;
    std::string img_path;   // View::s_Img_path = local_path / filename
};

std::vector<View> load_views(const char* path, std::string* root_path) {
    const std::string text = slurp(path);
    const Json doc = JsonParser(text).parse();
    SFM_REQUIRE(doc.kind == Json::Obj, SFM_ERR_INVALID_ARG, "%s: not a JSON object", path);
    if (root_path) {
        const Json* r = doc.get("root_path");
        *root_path = r && r->kind == Json::Str ? r->str : std::string();
    }
    const Json* views = doc.get("views");
    SFM_REQUIRE(views && views->kind == Json::Arr, SFM_ERR_INVALID_ARG, "%s: no \"views\" array", path);
    std::vector<View> out;
    for (const Json& kv : views->arr) {
        const Json* val = kv.get("value");
        SFM_REQUIRE(val, SFM_ERR_INVALID_ARG, "%s: view entry without \"value\"", path);
        const Json* f = view_fields(*val);
        SFM_REQUIRE(f, SFM_ERR_INVALID_ARG, "%s: view without filename/id_view", path);
        View v;
        v.id_view = as_u32(f->get("id_view"), "id_view");
        v.id_intrinsic = f->get("id_intrinsic") ? as_u32(f->get("id_intrinsic"), "id_intrinsic") : 0;
        v.id_pose = f->get("id_pose") ? as_u32(f->get("id_pose"), "id_pose") : 0;
        v.width = f->get("width") ? as_u32(f->get("width"), "width") : 0;
        v.height = f->get("height") ? as_u32(f->get("height"), "height") : 0;
        const Json* lp = f->get("local_path");
        const Json* fn = f->get("filename");
        SFM_REQUIRE(fn->kind == Json::Str, SFM_ERR_INVALID_ARG, "%s: filename is not a string", path);
        v.img_path = filespec(lp && lp->kind == Json::Str ? lp->str : std::string(), fn->str);
        out.push_back(std::move(v));
    }
    // Views is a Hash_Map keyed by id_view; iterate in id order
    std::sort(out.begin(), out.end(), [](const View& a, const View& b) { return a.id_view < b.id_view; });
    for (size_t k = 1; k < out.size(); ++k)
        SFM_REQUIRE(out[k].id_view != out[k - 1].id_view, SFM_ERR_INVALID_ARG, "%s: duplicate id_view %u", path,
                    out[k].id_view);
    return out;
}

// image_describer.json: the regions type must be 128-D uint8 SIFT
void check_describer(const char* path) {
    const std::string text = slurp(path);
    const Json doc = JsonParser(text).parse();
    const Json* rt = doc.get("regions_type");
    SFM_REQUIRE(rt, SFM_ERR_INVALID_ARG, "%s: no regions_type", path);
    const Json* name = rt->get("polymorphic_name");
    SFM_REQUIRE(name && name->kind == Json::Str, SFM_ERR_INVALID_ARG, "%s: regions_type without polymorphic_name",
                path);
    SFM_REQUIRE(name->str == "SIFT_Regions", SFM_ERR_UNSUPPORTED,
                "%s: regions type %s (this build matches 128-D uint8 SIFT_Regions)", path, name->str.c_str());
}

std::vector<uint8_t> read_desc(const char* path) {
    std::ifstream f(path, std::ios::binary);
    SFM_REQUIRE(f.good(), SFM_ERR_INVALID_ARG, "cannot open %s", path);
    uint64_t n = 0;
    f.read(reinterpret_cast<char*>(&n), 8);
    SFM_REQUIRE(f.gcount() == 8, SFM_ERR_INVALID_ARG, "%s: truncated header", path);
    SFM_REQUIRE(n < (1ull << 31), SFM_ERR_INVALID_ARG, "%s: implausible descriptor count %llu", path,
                (unsigned long long)n);
    std::vector<uint8_t> d(n * 128);
    if (n) f.read(reinterpret_cast<char*>(d.data()), (std::streamsize)d.size());
    SFM_REQUIRE(n == 0 || (size_t)f.gcount() == d.size(), SFM_ERR_INVALID_ARG, "%s: truncated (%llu descriptors)",
                path, (unsigned long long)n);
    return d;
}

std::vector<float> read_feat(const char* path) {
    std::ifstream f(path);
    SFM_REQUIRE(f.good(), SFM_ERR_INVALID_ARG, "cannot open %s", path);
    std::vector<float> v;
    float x, y, s, o;
    while (f >> x >> y >> s >> o) {
        v.push_back(x); v.push_back(y); v.push_back(s); v.push_back(o);
    }
    SFM_REQUIRE(f.eof(), SFM_ERR_INVALID_ARG, "%s: malformed feature line %zu", path, v.size() / 4 + 1);
    return v;
}

// loadPairs(N, file, pairs): each line "I J1 J2 ...", every (I, Jk) stored
// as (min, max) in a std::set; out-of-range or I == J is an error
std::set<std::pair<uint32_t, uint32_t>> load_pairs(const char* path, int64_t n_views) {
    std::ifstream f(path);
    SFM_REQUIRE(f.good(), SFM_ERR_INVALID_ARG, "cannot open %s", path);
    std::set<std::pair<uint32_t, uint32_t>> out;
    std::string line;
    int64_t ln = 0;
    while (std::getline(f, line)) {
        ++ln;
        std::istringstream ss(line);
        std::vector<int64_t> v;
        std::string tok;
        while (ss >> tok) {
            char* e = nullptr;
            const long long x = std::strtoll(tok.c_str(), &e, 10);
            SFM_REQUIRE(*e == '\0' && x >= 0, SFM_ERR_INVALID_ARG, "%s:%lld: bad index '%s'", path, (long long)ln,
                        tok.c_str());
            v.push_back(x);
        }
        SFM_REQUIRE(v.size() >= 2, SFM_ERR_INVALID_ARG, "%s:%lld: invalid input file", path, (long long)ln);
        for (size_t k = 1; k < v.size(); ++k) {
            SFM_REQUIRE(v[0] < n_views && v[k] < n_views, SFM_ERR_INVALID_ARG, "%s:%lld: index out of range", path,
                        (long long)ln);
            SFM_REQUIRE(v[0] != v[k], SFM_ERR_INVALID_ARG, "%s:%lld: pair with the same index", path, (long long)ln);
            out.insert({(uint32_t)std::min(v[0], v[k]), (uint32_t)std::max(v[0], v[k])});
        }
    }
    return out;
}

void save_pairs(const char* path, const std::vector<std::pair<uint32_t, uint32_t>>& pairs) {
    std::ofstream f(path);
    SFM_REQUIRE(f.good(), SFM_ERR_INVALID_ARG, "cannot write %s", path);
    for (const auto& p : pairs) f << p.first << ' ' << p.second << '\n';
    SFM_REQUIRE(!f.bad(), SFM_ERR_INVALID_ARG, "write failed: %s", path);
}

bool ext_is(const std::string& p, const char* ext) {
    const size_t d = p.find_last_of('.');
    return d != std::string::npos && p.compare(d + 1, std::string::npos, ext) == 0;
}

struct MatchSet {
    std::vector<std::pair<uint32_t, uint32_t>> pairs;
    std::vector<int64_t> counts;
    std::vector<uint32_t> i, j;
};

template <class T>
void put(std::ofstream& f, T v) {
    f.write(reinterpret_cast<const char*>(&v), sizeof v);   // little-endian host (x86-64)
}
template <class T>
T get(std::ifstream& f, const char* path) {
    T v{};
    f.read(reinterpret_cast<char*>(&v), sizeof v);
    SFM_REQUIRE(f.gcount() == (std::streamsize)sizeof v, SFM_ERR_INVALID_ARG, "%s: truncated", path);
    return v;
}

// pairs must be strictly increasing (std::map<Pair, IndMatches> order)
void save_matches(const char* path, const MatchSet& m) {
    for (size_t k = 1; k < m.pairs.size(); ++k)
        SFM_REQUIRE(m.pairs[k - 1] < m.pairs[k], SFM_ERR_INVALID_ARG, "matches: pairs not strictly increasing");
    const std::string p(path);
    if (ext_is(p, "txt")) {
        std::ofstream f(path);
        SFM_REQUIRE(f.good(), SFM_ERR_INVALID_ARG, "cannot write %s", path);
        int64_t off = 0;
        for (size_t k = 0; k < m.pairs.size(); ++k) {
            f << m.pairs[k].first << " " << m.pairs[k].second << '\n' << m.counts[k] << '\n';
            for (int64_t c = 0; c < m.counts[k]; ++c, ++off) f << m.i[off] << " " << m.j[off] << '\n';
        }
        SFM_REQUIRE(!f.bad(), SFM_ERR_INVALID_ARG, "write failed: %s", path);
        return;
    }
    SFM_REQUIRE(ext_is(p, "bin"), SFM_ERR_INVALID_ARG, "%s: matches files are .bin or .txt", path);
    std::ofstream f(path, std::ios::binary);
    SFM_REQUIRE(f.good(), SFM_ERR_INVALID_ARG, "cannot write %s", path);
    put<uint8_t>(f, 1);                            // PortableBinary: little endian
    put<uint64_t>(f, (uint64_t)m.pairs.size());    // map size tag
    int64_t off = 0;
    for (size_t k = 0; k < m.pairs.size(); ++k) {
        put<uint32_t>(f, m.pairs[k].first);
        put<uint32_t>(f, m.pairs[k].second);
        put<uint64_t>(f, (uint64_t)m.counts[k]);   // vector<IndMatch> size tag
        for (int64_t c = 0; c < m.counts[k]; ++c, ++off) {
            put<uint32_t>(f, m.i[off]);
            put<uint32_t>(f, m.j[off]);
        }
    }
    SFM_REQUIRE(!f.bad(), SFM_ERR_INVALID_ARG, "write failed: %s", path);
}

MatchSet load_matches(const char* path) {
    MatchSet m;
    const std::string p(path);
    if (ext_is(p, "txt")) {
        std::ifstream f(path);
        SFM_REQUIRE(f.good(), SFM_ERR_INVALID_ARG, "cannot open %s", path);
        uint64_t I, J, n;
        while (f >> I >> J >> n) {
            m.pairs.emplace_back((uint32_t)I, (uint32_t)J);
            m.counts.push_back((int64_t)n);
            for (uint64_t c = 0; c < n; ++c) {
                uint64_t a, b;
                SFM_REQUIRE((bool)(f >> a >> b), SFM_ERR_INVALID_ARG, "%s: truncated pair (%llu, %llu)", path,
                            (unsigned long long)I, (unsigned long long)J);
                m.i.push_back((uint32_t)a);
                m.j.push_back((uint32_t)b);
            }
        }
        SFM_REQUIRE(f.eof(), SFM_ERR_INVALID_ARG, "%s: malformed", path);
        return m;
    }
    std::ifstream f(path, std::ios::binary);
    SFM_REQUIRE(f.good(), SFM_ERR_INVALID_ARG, "cannot open %s", path);
    const uint8_t le = get<uint8_t>(f, path);
    SFM_REQUIRE(le == 1, SFM_ERR_UNSUPPORTED, "%s: big-endian portable archive", path);
    const uint64_t np = get<uint64_t>(f, path);
    for (uint64_t k = 0; k < np; ++k) {
        const uint32_t I = get<uint32_t>(f, path), J = get<uint32_t>(f, path);
        const uint64_t n = get<uint64_t>(f, path);
        SFM_REQUIRE(n < (1ull << 32), SFM_ERR_INVALID_ARG, "%s: implausible match count", path);
        m.pairs.emplace_back(I, J);
        m.counts.push_back((int64_t)n);
        for (uint64_t c = 0; c < n; ++c) {
            m.i.push_back(get<uint32_t>(f, path));
            m.j.push_back(get<uint32_t>(f, path));
        }
    }
    f.peek();
    SFM_REQUIRE(f.eof(), SFM_ERR_INVALID_ARG, "%s: trailing bytes", path);
    return m;
}

// IndMatchDecorator<float>::getDeduplicated (openMVG matching/
// indMatchDecoratorXY.hpp, un-vendored: SURVEY §8c) restated: every match is
// decorated with its keypoint coordinates (xI, yI, xJ, yJ) and the decorated
// list -- in (i, j) order, as IndMatch::getDeduplicated leaves it -- is copied
// into a std::set ordered by the decorator's operator<, whose iteration order
// is the output.  That comparator is not a strict weak order (x1 only picks
// which branch compares y1), so the survivors and their order are those of
// libstdc++'s set built from the range: the same container, comparator and
// insertion sequence as the reference's build, hence the same tree walk.
struct DecoratedMatch {
    float x1, y1, x2, y2;
    uint32_t i, j;
};
struct DecoratorLess {
    static bool same(const DecoratedMatch& a, const DecoratedMatch& b) {
        return a.x1 == b.x1 && a.y1 == b.y1 && a.x2 == b.x2 && a.y2 == b.y2;
    }
    bool operator()(const DecoratedMatch& a, const DecoratedMatch& b) const {
        if (same(a, b)) return false;
        if (a.x1 < b.x1) return a.y1 < b.y1;
        if (a.x1 > b.x1) return a.y1 < b.y1;
        return a.x2 < b.x2 && a.y2 < b.y2;
    }
};
void dedup_xy(std::vector<std::pair<uint32_t, uint32_t>>& v, const std::vector<float>& fi,
              const std::vector<float>& fj) {
    std::vector<DecoratedMatch> dec;
    dec.reserve(v.size());
    for (const auto& m : v)
        dec.push_back(DecoratedMatch{fi[4 * (size_t)m.first], fi[4 * (size_t)m.first + 1], fj[4 * (size_t)m.second],
                                     fj[4 * (size_t)m.second + 1], m.first, m.second});
    const std::set<DecoratedMatch, DecoratorLess> uniq(dec.begin(), dec.end());
    v.clear();
    for (const auto& d : uniq) v.emplace_back(d.i, d.j);
}

}  // namespace
}  // namespace sfm

using namespace sfm;

extern "C" int sfm_mvg_load_views(const char* path, sfm_mvg_view* views, int32_t cap, int32_t* n_views) {
    return guarded([&] {
        SFM_REQUIRE(path && n_views, SFM_ERR_INVALID_ARG, "null argument");
        const auto v = load_views(path, nullptr);
        *n_views = (int32_t)v.size();
        if (views) {
            SFM_REQUIRE(cap >= (int32_t)v.size(), SFM_ERR_INVALID_ARG, "views capacity %d < %zu", cap, v.size());
            for (size_t k = 0; k < v.size(); ++k) {
                SFM_REQUIRE(v[k].img_path.size() < sizeof(views[k].img_path), SFM_ERR_INVALID_ARG,
                            "image path too long: %s", v[k].img_path.c_str());
                views[k].id_view = v[k].id_view;
                views[k].id_intrinsic = v[k].id_intrinsic;
                views[k].id_pose = v[k].id_pose;
                views[k].width = v[k].width;
                views[k].height = v[k].height;
                std::memset(views[k].img_path, 0, sizeof(views[k].img_path));
                std::memcpy(views[k].img_path, v[k].img_path.data(), v[k].img_path.size());
            }
        }
        return SFM_OK;
    });
}

extern "C" int sfm_mvg_check_describer(const char* path) {
    return guarded([&] {
        SFM_REQUIRE(path, SFM_ERR_INVALID_ARG, "null argument");
        check_describer(path);
        return SFM_OK;
    });
}

extern "C" int sfm_mvg_read_desc(const char* path, uint8_t* desc, int64_t cap_rows, int64_t* n_rows) {
    return guarded([&] {
        SFM_REQUIRE(path && n_rows, SFM_ERR_INVALID_ARG, "null argument");
        const auto d = read_desc(path);
        *n_rows = (int64_t)(d.size() / 128);
        if (desc) {
            SFM_REQUIRE(cap_rows >= *n_rows, SFM_ERR_INVALID_ARG, "capacity %lld < %lld rows", (long long)cap_rows,
                        (long long)*n_rows);
            if (!d.empty()) std::memcpy(desc, d.data(), d.size());
        }
        return SFM_OK;
    });
}

extern "C" int sfm_mvg_write_desc(const char* path, const uint8_t* desc, int64_t n_rows) {
    return guarded([&] {
        SFM_REQUIRE(path && (desc || n_rows == 0) && n_rows >= 0, SFM_ERR_INVALID_ARG, "bad argument");
        std::ofstream f(path, std::ios::binary);
        SFM_REQUIRE(f.good(), SFM_ERR_INVALID_ARG, "cannot write %s", path);
        put<uint64_t>(f, (uint64_t)n_rows);
        if (n_rows) f.write(reinterpret_cast<const char*>(desc), (std::streamsize)(n_rows * 128));
        SFM_REQUIRE(!f.bad(), SFM_ERR_INVALID_ARG, "write failed: %s", path);
        return SFM_OK;
    });
}

extern "C" int sfm_mvg_read_feat(const char* path, float* xyso, int64_t cap_rows, int64_t* n_rows) {
    return guarded([&] {
        SFM_REQUIRE(path && n_rows, SFM_ERR_INVALID_ARG, "null argument");
        const auto v = read_feat(path);
        *n_rows = (int64_t)(v.size() / 4);
        if (xyso) {
            SFM_REQUIRE(cap_rows >= *n_rows, SFM_ERR_INVALID_ARG, "capacity %lld < %lld rows", (long long)cap_rows,
                        (long long)*n_rows);
            if (!v.empty()) std::memcpy(xyso, v.data(), v.size() * sizeof(float));
        }
        return SFM_OK;
    });
}

extern "C" int sfm_mvg_load_pairs(const char* path, int32_t n_views, int32_t* pairs, int64_t cap, int64_t* n_pairs) {
    return guarded([&] {
        SFM_REQUIRE(path && n_pairs && n_views >= 0, SFM_ERR_INVALID_ARG, "bad argument");
        const auto s = load_pairs(path, n_views);
        *n_pairs = (int64_t)s.size();
        if (pairs) {
            SFM_REQUIRE(cap >= *n_pairs, SFM_ERR_INVALID_ARG, "pairs capacity %lld < %lld", (long long)cap,
                        (long long)*n_pairs);
            int64_t k = 0;
            for (const auto& p : s) {
                pairs[2 * k] = (int32_t)p.first;
                pairs[2 * k + 1] = (int32_t)p.second;
                ++k;
            }
        }
        return SFM_OK;
    });
}

extern "C" int sfm_mvg_save_pairs(const char* path, const int32_t* pairs, int64_t n_pairs) {
    return guarded([&] {
        SFM_REQUIRE(path && (pairs || n_pairs == 0) && n_pairs >= 0, SFM_ERR_INVALID_ARG, "bad argument");
        std::set<std::pair<uint32_t, uint32_t>> s;   // Pair_Set
        for (int64_t k = 0; k < n_pairs; ++k) {
            SFM_REQUIRE(pairs[2 * k] >= 0 && pairs[2 * k + 1] >= 0, SFM_ERR_INVALID_ARG, "negative view index");
            s.insert({(uint32_t)pairs[2 * k], (uint32_t)pairs[2 * k + 1]});
        }
        save_pairs(path, std::vector<std::pair<uint32_t, uint32_t>>(s.begin(), s.end()));
        return SFM_OK;
    });
}

extern "C" int sfm_mvg_save_matches(const char* path, const int32_t* pairs, int64_t n_pairs, const int64_t* counts,
                                    const uint32_t* i, const uint32_t* j) {
    return guarded([&] {
        SFM_REQUIRE(path && n_pairs >= 0 && (n_pairs == 0 || (pairs && counts)), SFM_ERR_INVALID_ARG,
                    "bad argument");
        MatchSet m;
        int64_t total = 0;
        for (int64_t k = 0; k < n_pairs; ++k) {
            SFM_REQUIRE(counts[k] >= 0 && pairs[2 * k] >= 0 && pairs[2 * k + 1] >= 0, SFM_ERR_INVALID_ARG,
                        "bad pair %lld", (long long)k);
            m.pairs.emplace_back((uint32_t)pairs[2 * k], (uint32_t)pairs[2 * k + 1]);
            m.counts.push_back(counts[k]);
            total += counts[k];
        }
        SFM_REQUIRE(total == 0 || (i && j), SFM_ERR_INVALID_ARG, "null match arrays");
        m.i.assign(i, i + total);
        m.j.assign(j, j + total);
        save_matches(path, m);
        return SFM_OK;
    });
}

extern "C" int sfm_mvg_load_matches(const char* path, int32_t* pairs, int64_t* counts, uint32_t* i, uint32_t* j,
                                    int64_t cap_pairs, int64_t cap_matches, int64_t* n_pairs, int64_t* n_matches) {
    return guarded([&] {
        SFM_REQUIRE(path && n_pairs && n_matches, SFM_ERR_INVALID_ARG, "null argument");
        const MatchSet m = load_matches(path);
        *n_pairs = (int64_t)m.pairs.size();
        *n_matches = (int64_t)m.i.size();
        if (pairs || counts || i || j) {
            SFM_REQUIRE(cap_pairs >= *n_pairs && cap_matches >= *n_matches, SFM_ERR_INVALID_ARG,
                        "capacity too small");
            for (size_t k = 0; k < m.pairs.size(); ++k) {
                if (pairs) {
                    pairs[2 * k] = (int32_t)m.pairs[k].first;
                    pairs[2 * k + 1] = (int32_t)m.pairs[k].second;
                }
                if (counts) counts[k] = m.counts[k];
            }
            if (i) std::copy(m.i.begin(), m.i.end(), i);
            if (j) std::copy(m.j.begin(), m.j.end(), j);
        }
        return SFM_OK;
    });
}

// sparseBuilder::matchPair (sparseBuilder.cpp:758-807): pairs.bin of
// exhaustivePairs(#views) next to sfm_data.json
extern "C" int sfm_sparse_match_pair(const char* matches_dir) {
    return guarded([&] {
        SFM_REQUIRE(matches_dir, SFM_ERR_INVALID_ARG, "null argument");
        const std::string dir(matches_dir);
        const auto views = load_views(filespec(dir, "sfm_data.json").c_str(), nullptr);
        const uint32_t n = (uint32_t)views.size();
        std::vector<std::pair<uint32_t, uint32_t>> p;
        p.reserve((size_t)n * (n > 0 ? n - 1 : 0) / 2);
        for (uint32_t a = 0; a < n; ++a)
            for (uint32_t b = a + 1; b < n; ++b) p.emplace_back(a, b);
        save_pairs(filespec(dir, "pairs.bin").c_str(), p);
        return SFM_OK;
    });
}

// sparseBuilder::match (sparseBuilder.cpp:809-1023), file-staged: views from
// sfm_data.json, regions <stem>.desc / <stem>.feat, pairs from pairs.bin
// (exhaustive when the file is absent, :944-947), one resident matcher plan on
// the GPU, then matches.putative.bin (non-empty pairs only, as
// Matcher_Regions inserts them) and preemptive_pairs.txt.  An existing
// matches.putative.bin is reloaded instead unless opts->force (:890-900).
extern "C" int sfm_sparse_match(sfm_ctx* ctx, const char* matches_dir, const sfm_sparse_match_opts* opts,
                                sfm_sparse_match_stats* stats) {
    return guarded([&] {
        SFM_REQUIRE(ctx && matches_dir, SFM_ERR_INVALID_ARG, "null argument");
        // NULL opts: the reference's own settings, "AUTO" on SIFT regions ->
        // cascade hashing (:811-814,911-914), fDistRatio 0.8f, bForce false
        sfm_sparse_match_opts o{SFM_MATCH_CASCADE, 0.8f, 0, 1, {0, 0}};
        if (opts) o = *opts;
        SFM_REQUIRE(o.mode == SFM_MATCH_RATIO || o.mode == SFM_MATCH_MUTUAL || o.mode == SFM_MATCH_CASCADE,
                    SFM_ERR_INVALID_ARG, "bad mode %d", o.mode);
        sfm_sparse_match_stats st{};
        const std::string dir(matches_dir), out = filespec(dir, "matches.putative.bin");
        if (!o.force && is_file(out)) {
            const MatchSet m = load_matches(out.c_str());
            st.reloaded = 1;
            st.n_pairs_out = (int64_t)m.pairs.size();
            st.n_matches = (int64_t)m.i.size();
            if (stats) *stats = st;
            return SFM_OK;
        }
        std::string root;
        const auto views = load_views(filespec(dir, "sfm_data.json").c_str(), &root);
        check_describer(filespec(dir, "image_describer.json").c_str());
        // regions per view, keyed by id_view; plan rows in view order
        std::map<uint32_t, int32_t> slot;
        std::vector<uint8_t> desc;
        std::vector<int64_t> off(1, 0);
        std::vector<std::vector<float>> feats;
        for (const auto& v : views) {
            const std::string stem = basename_part(filespec(root, v.img_path));
            auto d = read_desc(filespec(dir, stem + ".desc").c_str());
            std::vector<float> f;
            if (o.dedup_xy) {
                f = read_feat(filespec(dir, stem + ".feat").c_str());
                SFM_REQUIRE(f.size() / 4 == d.size() / 128, SFM_ERR_INVALID_ARG,
                            "view %u: %zu features but %zu descriptors", v.id_view, f.size() / 4, d.size() / 128);
            }
            slot[v.id_view] = (int32_t)feats.size();
            desc.insert(desc.end(), d.begin(), d.end());
            off.push_back(off.back() + (int64_t)(d.size() / 128));
            feats.push_back(std::move(f));
        }
        std::set<std::pair<uint32_t, uint32_t>> pairs;
        const std::string pf = filespec(dir, "pairs.bin");
        // loadPairs(pairs.bin) failing is an error in the reference (:957-960)
        SFM_REQUIRE(is_file(pf), SFM_ERR_INVALID_ARG, "%s: no pairs file (run matchPair first)", pf.c_str());
        pairs = load_pairs(pf.c_str(), (int64_t)views.size());
        st.n_views = (int64_t)views.size();
        st.n_pairs_in = (int64_t)pairs.size();
        // pairs whose views have no regions are skipped by Matcher_Regions
        // (:continue); the cascade matcher keeps them, since every view of the
        // pair list enters its zero-mean descriptor (an empty one as zeros)
        std::vector<std::pair<uint32_t, uint32_t>> run;
        std::vector<int32_t> pv;
        for (const auto& p : pairs) {
            auto a = slot.find(p.first), b = slot.find(p.second);
            if (a == slot.end() || b == slot.end()) continue;
            if (o.mode != SFM_MATCH_CASCADE &&
                (off[a->second + 1] == off[a->second] || off[b->second + 1] == off[b->second]))
                continue;
            run.push_back(p);
            pv.push_back(a->second);
            pv.push_back(b->second);
        }
        MatchSet m;
        if (!run.empty()) {
            sfm_match_plan* plan = nullptr;
            int rc = sfm_match_plan_create(ctx, desc.data(), off.data(), (int32_t)views.size(), &plan);
            if (rc != SFM_OK) throw SfmError{rc};
            std::unique_ptr<sfm_match_plan, int (*)(sfm_match_plan*)> guard(plan, sfm_match_plan_destroy);
            sfm_match_options mo{o.mode, o.ratio};
            int64_t total = 0;
            rc = sfm_match_plan_run(plan, pv.data(), (int64_t)run.size(), &mo, &total);
            if (rc != SFM_OK) throw SfmError{rc};
            std::vector<int64_t> counts(run.size());
            std::vector<uint32_t> ii((size_t)std::max<int64_t>(total, 1)), jj(ii.size());
            std::vector<int32_t> dd(ii.size());
            rc = sfm_match_plan_fetch(plan, counts.data(), ii.data(), jj.data(), dd.data());
            if (rc != SFM_OK) throw SfmError{rc};
            int64_t k = 0;
            std::vector<std::pair<uint32_t, uint32_t>> v;
            for (size_t q = 0; q < run.size(); ++q) {
                v.clear();
                for (int64_t c = 0; c < counts[q]; ++c, ++k) v.emplace_back(ii[k], jj[k]);
                if (o.dedup_xy) dedup_xy(v, feats[slot[run[q].first]], feats[slot[run[q].second]]);
                if (v.empty()) continue;
                m.pairs.push_back(run[q]);
                m.counts.push_back((int64_t)v.size());
                for (const auto& x : v) {
                    m.i.push_back(x.first);
                    m.j.push_back(x.second);
                }
            }
        }
        save_matches(out.c_str(), m);
        save_pairs(filespec(dir, "preemptive_pairs.txt").c_str(), m.pairs);
        st.n_pairs_out = (int64_t)m.pairs.size();
        st.n_matches = (int64_t)m.i.size();
        if (stats) *stats = st;
        return SFM_OK;
    });
}

extern "C" int sfm_sparse_filter(sfm_ctx* ctx, const char* matches_dir, const sfm_fmatrix_opts* opts,
                                 sfm_sparse_filter_stats* stats) {
    return guarded([&] {
        SFM_REQUIRE(ctx && matches_dir, SFM_ERR_INVALID_ARG, "null argument");
        sfm_fmatrix_opts o{4.0, 2048, 0};   // GeometricFilter_FMatrix_AC(4.0, imax_iteration = 2048)
        if (opts) o = *opts;
        const std::string dir(matches_dir);
        std::string root;
        // Load(sfm_data, VIEWS | INTRINSICS) (:1095), putative matches (:1138)
        const auto views = load_views(filespec(dir, "sfm_data.json").c_str(), &root);
        std::map<uint32_t, size_t> vix;
        for (size_t k = 0; k < views.size(); ++k) vix[views[k].id_view] = k;
        const MatchSet put = load_matches(filespec(dir, "matches.putative.bin").c_str());
        std::map<size_t, std::vector<float>> feats;   // MatchesPairToMat: feature positions per view
        auto feat_of = [&](uint32_t id) -> const std::vector<float>& {
            auto it = vix.find(id);
            SFM_REQUIRE(it != vix.end(), SFM_ERR_INVALID_ARG, "matches reference view %u not in sfm_data.json", id);
            auto f = feats.find(it->second);
            if (f != feats.end()) return f->second;
            const std::string stem = basename_part(filespec(root, views[it->second].img_path));
            return feats[it->second] = read_feat(filespec(dir, stem + ".feat").c_str());
        };
        const int64_t np = (int64_t)put.pairs.size();
        std::vector<int64_t> off(np + 1, 0);
        std::vector<double> xy(4 * std::max<size_t>(put.i.size(), 1));
        std::vector<int32_t> wh(4 * std::max<int64_t>(np, 1));
        for (int64_t q = 0; q < np; ++q) {
            const auto& fi = feat_of(put.pairs[q].first);
            const auto& fj = feat_of(put.pairs[q].second);
            const View& vi = views[vix[put.pairs[q].first]];
            const View& vj = views[vix[put.pairs[q].second]];
            wh[4 * q] = (int32_t)vi.width; wh[4 * q + 1] = (int32_t)vi.height;
            wh[4 * q + 2] = (int32_t)vj.width; wh[4 * q + 3] = (int32_t)vj.height;
            off[q + 1] = off[q] + put.counts[q];
            for (int64_t k = off[q]; k < off[q + 1]; ++k) {
                const uint32_t a = put.i[k], b = put.j[k];
                SFM_REQUIRE((size_t)a < fi.size() / 4 && (size_t)b < fj.size() / 4, SFM_ERR_INVALID_ARG,
                            "pair (%u, %u): match (%u, %u) outside the features", put.pairs[q].first,
                            put.pairs[q].second, a, b);
                xy[4 * k] = fi[4 * (size_t)a];
                xy[4 * k + 1] = fi[4 * (size_t)a + 1];
                xy[4 * k + 2] = fj[4 * (size_t)b];
                xy[4 * k + 3] = fj[4 * (size_t)b + 1];
            }
        }
        std::vector<sfm_fmatrix_result> res((size_t)std::max<int64_t>(np, 1));
        std::vector<int32_t> inl(std::max<size_t>(put.i.size(), 1));
        if (np) {
            const int rc = sfm_fmatrix_ac(ctx, np, off.data(), xy.data(), wh.data(), &o, res.data(), inl.data());
            if (rc != SFM_OK) throw SfmError{rc};
        }
        // Robust_model_estimation keeps the pairs whose estimation succeeded,
        // each with putative[index] for index in vec_inliers order
        MatchSet out;
        for (int64_t q = 0; q < np; ++q) {
            if (res[q].n_inliers <= 0) continue;
            out.pairs.push_back(put.pairs[q]);
            out.counts.push_back(res[q].n_inliers);
            for (int32_t t = 0; t < res[q].n_inliers; ++t) {
                const int64_t k = off[q] + inl[off[q] + t];
                out.i.push_back(put.i[k]);
                out.j.push_back(put.j[k]);
            }
        }
        save_matches(filespec(dir, "matches.f.bin").c_str(), out);
        if (stats) {
            stats->n_pairs_in = np;
            stats->n_matches_in = (int64_t)put.i.size();
            stats->n_pairs_out = (int64_t)out.pairs.size();
            stats->n_matches_out = (int64_t)out.i.size();
        }
        return SFM_OK;
    });
}
