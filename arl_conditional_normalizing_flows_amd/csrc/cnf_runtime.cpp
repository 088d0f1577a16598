// cnf_runtime.cpp — plan execution and the C ABI of libcnf_hip.so (include/cnf.h).
//
// Executes the layer schedule of cFlow.call (conv_cINN_make_model.py:1723-1798) as a fixed
// sequence of k_conv / k_coupling / map launches on the caller's stream. All memory is the
// caller's (params, aux, workspace); the plan owns only its index tables.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>

#include "../../include/cnf.h"
#include "cnf_kernels.h"
#include "cnf_plan.h"

struct cnf_plan {
    cnf::Plan* p;
};

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

struct HipError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

void hip_check(hipError_t e, const char* what) {
    if (e != hipSuccess) throw HipError(std::string(what) + ": " + hipGetErrorString(e));
}

#define CNF_TRY try {
#define CNF_CATCH                                                   \
    }                                                               \
    catch (const std::invalid_argument& e) {                        \
        return fail(CNF_E_INVALID, e.what());                       \
    }                                                               \
    catch (const HipError& e) {                                     \
        return fail(CNF_E_HIP, e.what());                           \
    }                                                               \
    catch (const std::exception& e) {                               \
        return fail(CNF_E_STATE, e.what());                         \
    }                                                               \
    catch (...) {                                                   \
        return fail(CNF_E_STATE, "unknown error");                  \
    }

inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

}  // namespace

namespace cnf {

// error reporting for the entry points defined outside this file (cnf_transforms.hip)
int set_error(int code, const char* msg) { return fail(code, msg); }

// ----------------------------------------------------------------------------------------------
// debug options (cnf_flow_desc.debug_options)
// ----------------------------------------------------------------------------------------------
Options parse_options(const char* s) {
    Options o;
    if (s == nullptr) return o;
    struct Field {
        const char* name;
        int Options::*f;
    };
    static const Field fields[] = {{"NETLDS", &Options::netlds},           {"GC", &Options::gc},
                                   {"PW", &Options::pw},                   {"GENERIC", &Options::generic},
                                   {"LAYOUT", &Options::layout},           {"FUSE_COUPLING", &Options::fuse_coupling},
                                   {"LDS_BWD", &Options::lds_bwd},         {"TRAIN_ALT", &Options::train_alt},
                                   {"TRAIN_SCHED", &Options::train_sched}};
    std::string str(s);
    size_t pos = 0;
    while (pos < str.size()) {
        size_t end = str.find(',', pos);
        if (end == std::string::npos) end = str.size();
        const std::string item = str.substr(pos, end - pos);
        pos = end + 1;
        if (item.empty()) continue;
        const size_t eq = item.find('=');
        if (eq == std::string::npos) throw std::invalid_argument("debug_options: expected NAME=VALUE, got '" + item + "'");
        const std::string key = item.substr(0, eq), val = item.substr(eq + 1);
        char* endp = nullptr;
        const long v = std::strtol(val.c_str(), &endp, 10);
        if (val.empty() || *endp != '\0') throw std::invalid_argument("debug_options: bad value in '" + item + "'");
        bool found = false;
        for (const Field& f : fields)
            if (key == f.name) {
                o.*(f.f) = (int)v;
                found = true;
            }
        if (!found) throw std::invalid_argument("debug_options: unknown option '" + key + "'");
    }
    if (o.lds_bwd < 0 || o.lds_bwd > 2) throw std::invalid_argument("debug_options: LDS_BWD is 0, 1 or 2");
    return o;
}

namespace {
thread_local const Options* g_opts = nullptr;
const Options kDefaultOptions{};
}  // namespace
const Options& opts() { return g_opts != nullptr ? *g_opts : kDefaultOptions; }
OptScope::OptScope(const Options* o) : prev(g_opts) {
    if (o != nullptr) g_opts = o;
}
OptScope::~OptScope() { g_opts = prev; }

LaunchTiming& launch_timing() {
    thread_local LaunchTiming t;
    return t;
}

// ----------------------------------------------------------------------------------------------
// geometry
// ----------------------------------------------------------------------------------------------
struct Geo {
    int TH, tiles, MR;
};

static Geo conv_geo(int h, int w) {
    Geo g;
    g.MR = (h * w >= 1024) ? 2 : 1;
    const int pt = 64 * g.MR;
    if (w > pt) throw std::invalid_argument("image width too large for the row-band tiling (w > 128)");
    g.TH = std::min(h, std::max(1, pt / w));
    g.tiles = (h + g.TH - 1) / g.TH;
    return g;
}

static int lds_stride(int cin) {  // pixel stride in floats, == 2 (mod 4): conflict-free A reads
    int s = std::max(cin, 2);
    while (s % 4 != 2) s++;
    return s;
}

struct ConvGeom1 {
    int MR, P, tiles;
};
static ConvGeom1 conv1_geo(int h, int w) {
    ConvGeom1 g;
    const int hw = h * w;
    g.MR = (hw >= 1024) ? 2 : 1;
    g.P = 64 * g.MR;
    g.tiles = (hw + g.P - 1) / g.P;
    return g;
}

// log-det partial slots (= k_coupling workgroups) per image: one per 64 compressed pixels, so the
// largest layers run one element per thread (latency-bound otherwise)
static int ld_parts_for(int npx) { return std::max(1, std::min(16, (npx + 63) / 64)); }

static uint32_t udiv_magic_host(uint32_t d) { return d <= 1 ? 0u : 0xFFFFFFFFu / d + 1u; }   // cnf_device.h udiv

WsLayout Plan::layout(int B) const {
    WsLayout L;
    int64_t n_uv = (int64_t)desc.io_h * desc.io_w * desc.io_d;
    int64_t n_u1c = 0, n_y = 0, n_t2 = 0, n_so = 0;
    int parts = 1, ldp = 1;
    for (const auto& c : couplings) {
        int64_t npx = (int64_t)c.hc * c.wc;
        n_u1c = std::max<int64_t>(n_u1c, npx * c.dc1);
        n_y = std::max<int64_t>(n_y, npx * c.nk);
        n_t2 = std::max<int64_t>(n_t2, npx * c.gc);
        n_so = std::max<int64_t>(n_so, npx * c.dc2);
        Geo g = conv_geo(c.hc, c.wc);
        parts = std::max(parts, 4 * g.tiles * (int)c.br.size());   // 4 waves per workgroup
        parts = std::max(parts, 4 * conv1_geo(c.hc, c.wc).tiles);
        parts = std::max(parts, 4 * ((c.hc * c.wc + 63) / 64));   // k_pw
        parts = std::max(parts, (int)c.br.size() * std::max(4 * g.tiles, 4 * ((c.hc * c.wc + 63) / 64)));   // mixed branches
        if (c.gc_fused) {   // k_gc groups' slots, then the tap-mode / k_conv<3> branches' after them
            int gp = 0, ing = 0;
            for (const auto& gg : c.gcg) {
                gp += GC_NW_MAX * gg.tiles();
                ing += (int)gg.br.size();
            }
            const int rest = (int)c.br.size() - ing;
            gp += rest * std::max(4 * g.tiles, 4 * ((c.hc * c.wc + 63) / 64));
            parts = std::max(parts, gp);
        }
        ldp = std::max(ldp, ld_parts_for((int)npx));
    }
    L.n_uv = n_uv;
    L.n_u1c = n_u1c;
    L.n_y = n_y;
    L.n_t2 = n_t2;
    L.n_so = n_so;
    L.st_parts = parts;
    L.ld_parts = ldp;
    size_t off = 0;
    auto take = [&](size_t bytes) {
        size_t o = off;
        off = align_up(off + bytes, 256);
        return o;
    };
    const size_t Bz = (size_t)B;
    L.uv[0] = take(Bz * n_uv * 4);
    L.uv[1] = take(Bz * n_uv * 4);
    L.u1c = take(Bz * n_u1c * 4);
    for (int n = 0; n < 2; n++) {
        L.y[n] = take(Bz * n_y * 4);
        L.t1[n] = take(Bz * n_y * 4);
        L.t2[n] = take(Bz * n_t2 * 4);
        L.so[n] = take(Bz * n_so * 4);
        L.so_alt[n] = take(Bz * n_so * 4);
        for (int k = 0; k < 3; k++) {   // LN slabs y, t1, t2: per-wave partials
            L.st_part[n][k] = take(Bz * parts * LNP * 4);
        }
    }

    L.ld = take(std::max<size_t>(1, couplings.size()) * Bz * ldp * 8);
    L.total = off;
    return L;
}

// ----------------------------------------------------------------------------------------------
// launch helpers
// ----------------------------------------------------------------------------------------------
struct Exec {
    Plan& p;
    const float* params;
    const float* aux;
    char* ws;
    WsLayout L;
    int B;
    hipStream_t st;

    template <class T>
    T* at(size_t off) const {
        return reinterpret_cast<T*>(ws + off);
    }

    void record(const std::string& name, double flops, double bytes, std::function<void(void*)> fn) {
        if (p.dry) {
            p.dry_launches.push_back(name);
            return;
        }
        const size_t k = p.recorded.size();
        const bool timed = p.timing && p.record && name.rfind("k_", 0) == 0;   // kernels only (not copies)
        if (timed) {
            while (p.ev.size() < 2 * (k + 1)) {
                hipEvent_t e;
                if (hipEventCreate(&e) != hipSuccess) throw std::runtime_error("hipEventCreate");
                p.ev.push_back(e);
            }
            launch_timing() = LaunchTiming{p.ev[2 * k], p.ev[2 * k + 1]};
        }
        try {
            fn(st);
        } catch (...) {
            launch_timing() = LaunchTiming{};
            throw;
        }
        // timed only when exactly one kernel wrote the pair (a launch helper may issue none)
        const bool wrote = timed && launch_timing().used == 1;
        launch_timing() = LaunchTiming{};
        if (p.record) {
            Recorded r;
            r.name = name;
            r.flops = flops;
            r.bytes = bytes;
            r.relaunch = std::move(fn);
            r.timed = wrote;
            p.recorded.push_back(std::move(r));
        }
    }
};

// LN statistics slab of one tensor: per-wave partials [B][st_parts][LNP] of which the last producer
// wrote the first nparts (see ConvProb)
struct Slab {
    float* part = nullptr;
    int nparts = 0;
};

struct ProbSpec {
    const float* in;
    int in_cs, in_off, cin;
    Slab in_st;               // input LN partials (.part == null: no LN)
    const float* gamma;
    const float* beta;
    int act;
    const float* wt;
    const float* bias;
    float* out;
    int out_cs, out_off, cout;
    const float* res;
    Slab out_st;              // .part == null: no output statistics
    int out_part_base;        // first partial slot of this problem
    int dil;
    float* out2 = nullptr;    // k_pw only: every output channel also to a plain [B][HW][cout] tensor
};

static const char* role_name(int r) {
    switch (r) {
        case ROLE_CONV_IN: return "conv_in";
        case ROLE_CONV_A: return "conv_a";
        case ROLE_GC: return "gc";
        case ROLE_CONV_B: return "conv_b";
        default: return "conv_out";
    }
}

static uint32_t magic_for(int d, int64_t xmax) {
    // x / d == umulhi(x, ceil(2^32 / d)) exactly while x * d * d < 2^32 (error term x*e/2^32 < 1/d)
    if (d <= 1) return 0;
    if ((double)xmax * d * d >= 4294967296.0) throw std::invalid_argument("magic division out of range");
    return (uint32_t)((((uint64_t)1 << 32) + (uint64_t)d - 1) / (uint64_t)d);
}

// tap-mode source of a k_pw launch (streamed conv_in): the probs' `in` is the raw layer input u, the
// A operand the 3x3 im2col row over the mask-compressed half (K = 9 * dc), gathered in the kernel
struct TapSrc {
    int mask, W, D, dc, img;   // mask, full-res width / depth, channels per tap, floats per image of u
    int dil = 1, off = 0;      // mask < 0: plain NHWC source (D channels), taps from channel off, dilation
};

// returns the LN-partial slots per image each problem writes (4 per workgroup tile)
static int conv_launch(Exec& E, int ks, int role, int h, int w, const std::vector<ProbSpec>& probs,
                       uint64_t store_mask = ~0ull, const TapSrc* tap = nullptr, const int* st_map = nullptr,
                       const int* in_map = nullptr, bool* dual_done = nullptr) {
    const bool st_compact = st_map != nullptr;
    if (probs.empty()) return 0;
    if ((int)probs.size() > MAXPROB) throw std::invalid_argument("too many problems in one conv launch");
    ConvArgs a;
    std::memset(&a, 0, sizeof(a));
    a.H = h;
    a.W = w;
    a.nprob = (int)probs.size();
    a.B = E.B;
    Geo g{0, 0, 0};
    ConvGeom1 g1{0, 0, 0};
    if (ks == 3) {
        g = conv_geo(h, w);
        a.TH = g.TH;
        a.tiles_per_img = g.tiles;
    } else {
        g1 = conv1_geo(h, w);
        a.P = g1.P;
        a.tiles_per_img = g1.tiles;
    }
    size_t lds = 0;
    double flops = 0, bytes = 0;
    const double HWB = (double)h * w * E.B;
    bool vec = true;
    int pw_nr = 0, pw_gm = 0;
    for (size_t i = 0; i < probs.size(); i++) {
        const ProbSpec& s = probs[i];
        ConvProb& q = a.p[i];
        q.in = s.in;
        q.in_part = s.in_st.part;
        q.in_nparts = s.in_st.nparts;
        q.gamma = s.gamma;
        q.beta = s.beta;
        q.wt = s.wt;
        q.bias = s.bias;
        q.res = s.res;
        q.out = s.out;
        q.out_part = s.out_st.part;
        q.in_cs = s.in_cs;
        q.in_off = s.in_off;
        q.cin = s.cin;
        q.out_cs = s.out_cs;
        q.out_off = s.out_off;
        q.cout = s.cout;
        q.part_stride = E.L.st_parts;
        q.out_part_base = s.out_part_base;
        q.dil = s.dil;
        q.act = s.act;
        q.st_mask_lo = (uint32_t)(store_mask & 0xffffffffull);
        q.st_mask_hi = (uint32_t)(store_mask >> 32);
        q.st_compact = st_compact ? 1 : 0;
        q.st_map = st_map;
        q.in_mapped = in_map != nullptr ? 1 : 0;
        q.in_map = in_map;
        q.out2 = s.out2;
        if (in_map != nullptr && (ks != 1 || tap != nullptr || s.in_off != 0 || s.cin % 4 != 0))
            throw std::logic_error("mapped input: plain k_pw over whole quads only");
        if (st_compact && (s.res != nullptr || s.cout > 64)) throw std::logic_error("mapped stores: no residual, <= 64 outputs");
        if (s.cout > 64) throw std::invalid_argument("conv with more than 64 output channels");
        const int K = ks * ks * s.cin;
        q.nr = (s.cout + 15) / 16;
        size_t off = 128;
        if (ks == 3) {
            q.S = lds_stride(s.cin);
            q.Kpad = (K + 3) / 4 * 4;
            q.NS = 16 * q.nr;
            if (q.NS % 32 == 0) q.NS += 16;
            const int d = s.dil;
            const int WP = w + 2 * d;
            const int SR = g.TH + 2 * d;
            const int64_t total = (int64_t)SR * WP * s.cin;
            q.cin_mag = magic_for(s.cin, total + 256 * 4);
            q.wp_mag = magic_for(WP, (int64_t)SR * WP + 256 * 4);
            if (WP == 1) throw std::invalid_argument("degenerate width");
            size_t lin_f = (size_t)SR * WP * q.S;
            q.lds_in_off = (int)off;
            off = align_up(off + lin_f * 4, 16);
            q.lds_w_off = (int)off;
            off = align_up(off + (size_t)q.Kpad * q.NS * 4, 16);
            q.lds_k_off = (int)off;
            off = align_up(off + (size_t)q.Kpad * 4, 16);
        } else {
            const int G = (s.cin + 15) / 16;
            if (off < 512) off = 512;   // k_pw keeps its per-image LN table at bytes [256, 384)
            q.lds_w_off = (int)off;
            // k_pw stages the weights as the three bf16 planes of 32-deep K steps (1 KiB per plane, step and
            // 16-column block); k_conv1 reads the fp32 image, G x 16 x 16 x nr floats, which fits in it
            const size_t wx6 = (size_t)((s.cin + 31) / 32) * 3 * q.nr * 1024;
            off = align_up(off + std::max(wx6, (size_t)G * 16 * 16 * q.nr * 4), 16);
            // k_pw loads every channel quad the input window starts with 16 bytes at a time: a window
            // that is not quad-aligned (conv_b over the 62- / 30-channel concat of cfg5's grouped
            // stages) reads past its last channel into the next pixel (or 0 past the image), which
            // meets zero weight rows (the packed image pads K with zeros)
            pw_nr = std::max(pw_nr, q.nr);
            pw_gm = std::max(pw_gm, G);
        }
        lds = std::max(lds, off);
        flops += 2.0 * HWB * K * s.cout;
        // output bytes count only the stored channels (conv_a stores just the grouped branches' inputs)
        const uint64_t cmask = s.cout >= 64 ? ~0ull : ((1ull << s.cout) - 1);
        const double stored = (double)__builtin_popcountll(store_mask & cmask);
        bytes += 4.0 * (HWB * (tap ? tap->dc : s.cin) + HWB * (stored + (s.res ? s.cout : 0)) +
                        (s.in_st.part ? 2.0 * h * w * (tap ? tap->dc : s.cin) : 0.0) +
                        (double)K * s.cout + s.cout);
    }
    if (lds > 160 * 1024) throw std::invalid_argument("conv tile exceeds the 160 KiB LDS budget");
    if (ks == 1)   // k_pw stages every problem's weights as pw_nr column blocks: the workgroup's LDS covers them
        for (int i = 0; i < a.nprob; i++)
            if ((size_t)a.p[i].lds_w_off + (size_t)((a.p[i].cin + 31) / 32) * 3 * pw_nr * 1024 > lds || a.p[i].nr != pw_nr)
                throw std::logic_error("k_pw launch: problems of different widths or LDS short of the weight planes");
    const int ilds = (int)lds;
    if (pw_gm > 0) pw_gm = pw_gm <= 1 ? 1 : pw_gm <= 2 ? 2 : pw_gm <= 4 ? 4 : pw_gm <= 8 ? 8 : 0;
    bool ln_uniform = true;
    for (const ProbSpec& s : probs)
        ln_uniform = ln_uniform && ((s.in_st.part != nullptr) == (probs[0].in_st.part != nullptr)) &&
                     ((s.res != nullptr) == (probs[0].res != nullptr));
    bool fits32 = true;   // k_pw addresses one image per buffer resource with 32-bit byte offsets
    for (const ProbSpec& s : probs)
        fits32 = fits32 && (double)h * w * std::max(s.in_cs, s.out_cs) * 4.0 < 2147483648.0 &&
                 (tap == nullptr || (double)tap->img * 4.0 < 2147483648.0);
    const bool pw_ok = ks == 1 && vec && pw_gm > 0 && ln_uniform && fits32 && E.p.use_pw;
    if ((st_compact || in_map != nullptr) && !pw_ok) throw std::logic_error("mapped loads / stores need the k_pw path");
    if (dual_done != nullptr) *dual_done = pw_ok;   // (the other kernels ignore out2)
    if (!pw_ok)
        for (int i = 0; i < a.nprob; i++) a.p[i].out2 = nullptr;
    if (ks == 3) {
        const int grid_x = E.B * g.tiles;
        const int mr = g.MR;
        std::string name = std::string("k_conv3<") + std::to_string(mr) + "," + role_name(role) + ">";
        E.record(name, flops, bytes, [mr, role, a, grid_x, ilds](void* st) {
            launch_conv(3, mr, role, a, grid_x, ilds, (hipStream_t)st);
        });
        return 4 * g.tiles;
    } else if (pw_ok) {
        // k_pw: 64-pixel tiles (4 waves x 16 pixels), each workgroup looping over ipw images, sized
        // so the launch is one round of two workgroups per CU (see cnf_stream.hip)
        const bool resf = probs[0].res != nullptr;
        const int nw = 4;
        const int tiles = (h * w + 16 * nw - 1) / (16 * nw);
        a.tiles_per_img = tiles;
        for (int i = 0; i < a.nprob; i++) a.p[i].out_part_base = probs[i].out_part_base;
        const int64_t units = (int64_t)tiles * a.nprob * E.B;
        const bool lnf = probs[0].in_st.part != nullptr;
        a.ipw = (int)std::min<int64_t>(16, std::max<int64_t>(1, (units + 511) / 512));
#ifdef CNF_DIAG   // diagnostics: images per workgroup of the residual (conv_b) / other k_pw launches
        if (const char* e = std::getenv(resf ? "CNF_PW_IPW_RES" : "CNF_PW_IPW")) a.ipw = std::atoi(e);
#endif
        const int grid_x = tiles * ((E.B + a.ipw - 1) / a.ipw);
        const int nr = pw_nr, gm = pw_gm;
        const bool tapf = tap != nullptr;
        if (tap) {
            a.umask = tap->mask;
            a.uW = tap->W;
            a.uD = tap->D;
            a.udc = tap->dc;
            a.uimg = tap->img;
            a.udil = tap->dil;
            a.uoff = tap->off;
        }
        if (E.p.dry) {
            PwShape sh;
            if (pw_shape_of(nr, gm, lnf, resf, tapf, a, sh)) {
                bool seen = false;
                for (const PwShape& o : E.p.pw_shapes) seen = seen || std::memcmp(&o, &sh, sizeof(sh)) == 0;
                if (!seen) E.p.pw_shapes.push_back(sh);
            }
        }
        std::string name = std::string("k_pw<") + std::to_string(nr) + "," + std::to_string(gm) + "," +
                           role_name(role) + ">";
        E.record(name, flops, bytes, [nr, gm, lnf, resf, tapf, a, grid_x, ilds](void* st) {
            launch_pw(nr, gm, lnf, resf, tapf, a, grid_x, ilds, (hipStream_t)st);
        });
        return nw * tiles;
    } else {
        const int grid_x = E.B * g1.tiles;
        const int mr = g1.MR;
        std::string name = std::string("k_conv1<") + std::to_string(mr) + "," + (vec ? "vec" : "scalar") + "," +
                           role_name(role) + ">";
        E.record(name, flops, bytes, [mr, vec, role, a, grid_x, ilds](void* st) {
            launch_conv1(mr, vec, role, a, grid_x, ilds, (hipStream_t)st);
        });
        return 4 * g1.tiles;
    }
}

// tap-decomposed 3x3 (dilation 1, cout <= 7): see k_convtap
static void convtap_launch(Exec& E, int h, int w, const std::vector<ProbSpec>& probs) {
    ConvArgs a;
    std::memset(&a, 0, sizeof(a));
    Geo g = conv_geo(h, w);
    a.H = h;
    a.W = w;
    a.TH = g.TH;
    a.tiles_per_img = g.tiles;
    a.nprob = (int)probs.size();
    a.B = E.B;
    const int nband = (g.TH + 2) * w;
    int mt = (nband + 63) / 64;
    if (mt == 5) mt = 6;
    if (mt > 6) throw std::invalid_argument("tap conv band too large");
    size_t lds = 0;
    double flops = 0, bytes = 0;
    const double HWB = (double)h * w * E.B;
    bool vec = true;
    int pw_nr = 0, pw_gm = 0;
    for (size_t i = 0; i < probs.size(); i++) {
        const ProbSpec& s = probs[i];
        ConvProb& q = a.p[i];
        q.in = s.in;
        q.in_part = s.in_st.part;
        q.in_nparts = s.in_st.nparts;
        q.part_stride = E.L.st_parts;
        q.gamma = s.gamma;
        q.beta = s.beta;
        q.wt = s.wt;
        q.bias = s.bias;
        q.out = s.out;
        q.in_cs = s.in_cs;
        q.in_off = s.in_off;
        q.cin = s.cin;
        q.out_cs = s.out_cs;
        q.out_off = s.out_off;
        q.cout = s.cout;
        q.act = s.act;
        q.dil = 1;
        q.st_mask_lo = q.st_mask_hi = 0xffffffffu;
        if (9 * s.cout > 64) throw std::invalid_argument("tap conv needs 9*cout <= 64");
        q.nr = (9 * s.cout + 15) / 16;
        const int NSJ = 16 * q.nr;
        const int G = (s.cin + 15) / 16;
        size_t off = 128;
        q.lds_w_off = (int)off;
        off = align_up(off + (size_t)G * 16 * NSJ * 4, 16);
        q.lds_in_off = (int)off;
        off = align_up(off + (size_t)nband * (NSJ + 1) * 4, 16);
        q.lds_k_off = (int)off;
        off = align_up(off + (size_t)NSJ * 4, 16);
        lds = std::max(lds, off);
        if (s.cin % 4 || s.in_cs % 4 || s.in_off % 4) vec = false;
        flops += 2.0 * HWB * 9 * s.cin * s.cout;
        bytes += 4.0 * (HWB * s.cin + HWB * s.cout + (s.in_st.part ? 2.0 * h * w * s.cin : 0.0) + 9.0 * s.cin * s.cout);
    }
    if (lds > 160 * 1024) throw std::invalid_argument("tap conv exceeds the LDS budget");
    const int ilds = (int)lds, grid_x = E.B * g.tiles;
    std::string name = std::string("k_convtap<") + std::to_string(mt) + (vec ? ",vec" : ",scalar") + ",conv_out>";
    E.record(name, flops, bytes, [mt, vec, a, grid_x, ilds](void* st) {
        launch_convtap(mt, vec, a, grid_x, ilds, (hipStream_t)st);
    });
}

// k_net_lds geometry for coupling c; returns the LDS bytes (0 if the layer cannot use it)
static size_t netlds_setup(const Plan& p, const Coupling& c, NetLdsArgs& a) {
    std::memset(&a, 0, sizeof(a));
    if ((int)c.br.size() > NETLDS_MAXBR) return 0;
    for (const Branch& b : c.br)
        if (b.dil > 16) return 0;
    const int HW = c.hc * c.wc;
    a.H = c.H;
    a.W = c.W;
    a.D = c.D;
    a.mask = c.mask;
    a.hc = c.hc;
    a.wc = c.wc;
    a.dc1 = c.dc1;
    a.dc2 = c.dc2;
    a.nk = c.nk;
    a.gc = c.gc;
    a.R = c.R;
    a.nbr = (int)c.br.size();
    a.ln = p.desc.layer_norm;
    for (int i = 0; i < a.nbr; i++) {
        a.br_cin_off[i] = c.br[i].cin_off;
        a.br_cin[i] = c.br[i].cin;
        a.br_cout[i] = c.br[i].cout;
        a.br_out_off[i] = c.br[i].out_off;
        a.br_dil[i] = c.br[i].dil;
    }
    {   // disjoint union of the grouped branches' input channel windows (normalised once, in place)
        std::vector<std::pair<int, int>> iv;
        for (const Branch& b : c.br) iv.push_back({b.cin_off, b.cin_off + b.cin});
        std::sort(iv.begin(), iv.end());
        std::vector<std::pair<int, int>> mg;
        for (auto& x : iv) {
            if (!mg.empty() && x.first <= mg.back().second)
                mg.back().second = std::max(mg.back().second, x.second);
            else
                mg.push_back(x);
        }
        if ((int)mg.size() > NETLDS_MAXBR) return 0;
        a.nwin = (int)mg.size();
        for (int i = 0; i < a.nwin; i++) {
            a.win_off[i] = mg[i].first;
            a.win_len[i] = mg[i].second - mg[i].first;
        }
    }
    a.offs_per_net = c.lds_offs_per_net;
    const NetLdsGeom& g = c.lds;
    a.sy = g.sy;
    a.s1 = g.s1;
    a.s2 = g.s2;
    a.su = g.su;
    const NetParams& n0 = c.net[0];
    auto desc = [](const PackedConv& pc) { return LdsConv{pc.fmt, (int)pc.size, pc.kpad, pc.ns}; };
    a.ci = desc(n0.ci);
    a.co = desc(n0.co);
    if (!n0.rb.empty()) {
        a.ca = desc(n0.rb[0].ca);
        a.cb = desc(n0.rb[0].cb);
        for (int i = 0; i < a.nbr; i++) a.gcv[i] = desc(n0.rb[0].gc[i]);
    }
    a.off_y = g.off_y;
    a.off_t1 = g.off_t1;
    a.off_t2 = g.off_t2;
    a.off_w = g.off_w;
    a.off_k = g.off_k;
    a.off_ks = g.off_ks;
    auto nr = [](int cout) { return (cout + 15) / 16; };
    // the tap-decomposed conv_out runs in chunks of at most two 16-column blocks
    a.maxnr = std::max(nr(c.nk), c.co_fmt == PK_TAP ? std::min(2, nr(9 * c.dc2)) : nr(c.dc2));
    for (const Branch& b : c.br) a.maxnr = std::max(a.maxnr, nr(b.cout));
#ifdef CNF_DIAG
    if (const char* e = std::getenv("CNF_NETLDS_DUMP")) {   // diagnostics: every shape field, as C
        if (std::atoi(e)) {
            const int* w = reinterpret_cast<const int*>(&a.offs_per_net);
            const int n = (int)((reinterpret_cast<const char*>(&a.zero_bias) - reinterpret_cast<const char*>(w)) / 4);
            std::fprintf(stderr, "NETSHAPE hc=%d wc=%d mask=%d:", c.hc, c.wc, c.mask);
            for (int i = 0; i < n; i++) std::fprintf(stderr, " %d", w[i]);
            const int* w2 = reinterpret_cast<const int*>(&a.off_y);
            for (int i = 0; i < 7; i++) std::fprintf(stderr, " %d", w2[i]);
            std::fprintf(stderr, "\n");
        }
    }
    if (const char* e = std::getenv("CNF_NETLDS_VERBOSE"))
        if (std::atoi(e)) std::fprintf(stderr, "netlds layer hc=%d wc=%d nk=%d dc2=%d co_fmt=%d maxnr=%d\n", c.hc, c.wc,
                                       c.nk, c.dc2, c.co_fmt, a.maxnr);
#endif
    return (size_t)g.bytes;
}

static double net_flops(const Coupling& c) {
    const double HW = (double)c.hc * c.wc;
    double f = 9.0 * c.dc1 * c.nk + 9.0 * c.nk * c.dc2;
    double rb = (double)c.nk * c.nk + (double)c.gc * c.nk;
    for (const Branch& b : c.br) rb += 9.0 * b.cin * b.cout;
    return 2.0 * HW * (f + c.R * rb);
}

// One coupling layer: u -> v. dir=+1 forward (ld_part may collect Σs), dir=-1 inverse.
// pend: the previous layer's deferred coupling, applied by this layer's k_net_lds (forward, LDS
// layers only). defer: leave this layer's own coupling pending (no k_coupling launch) and describe it
// in *out_pend for the next layer's k_net_lds (the caller allows it only when that layer is an LDS
// layer of the same forward).
// save / so_save (training forward of a layer with the fused LDS backward): k_net_lds also writes the
// raw activations and LN statistics to save (LdsSave blocks) and its s / t outputs to so_save[2]
// nz (first coupling of cnf_flow_forward_noise, k_net_lds layers only): u is the noisy-input buffer,
// written by this layer's k_net_lds from nz->src (the fused gather)
static void run_coupling(Exec& E, const Coupling& c, const float* u, float* v, double* ld_part, int dir,
                         const CoupPend* pend = nullptr, bool defer = false, CoupPend* out_pend = nullptr,
                         float* save = nullptr, float* const* so_save = nullptr,
                         const TrainLayout::StreamSave* ss = nullptr, const InputPrepArgs* nz = nullptr) {
    const int B = E.B;
    const WsLayout& L = E.L;
    const float* P = E.params;
    const float* X = E.aux;
    const int nt3 = conv_geo(c.hc, c.wc).tiles;     // LN partials written by a 3x3 launch (per problem)
    const int nt1 = conv1_geo(c.hc, c.wc).tiles;    // ... by a 1x1 launch
    const int nbr = (int)c.br.size();
    const bool ln = E.p.desc.layer_norm != 0;
    // k_net_lds layers alternate between two s/t sets by coupling index, so a layer applying its
    // predecessor's deferred coupling never writes the set it reads
    const bool alt = c.use_lds && (c.index & 1) != 0;
    float* so0 = so_save ? so_save[0] : E.at<float>(alt ? L.so_alt[0] : L.so[0]);
    float* so1 = so_save ? so_save[1] : E.at<float>(alt ? L.so_alt[1] : L.so[1]);
    if (save != nullptr && (!c.use_lds || so_save == nullptr || defer))
        throw std::logic_error("training save: k_net_lds layers without a deferred law only");
    if ((pend != nullptr || defer) && !c.use_lds)
        throw std::logic_error("deferred couplings are only fused into k_net_lds layers");
    if (pend != nullptr && pend->dir != dir) throw std::logic_error("deferred coupling of the other direction");
    const float* tap_c[2] = {nullptr, nullptr};   // streamed tap-GEMM conv_out (finished in k_coupling)
    const float* tap_b[2] = {nullptr, nullptr};
    NetLdsArgs na;
    const size_t nlds = c.use_lds ? netlds_setup(E.p, c, na) : 0;
    if (c.use_lds && nlds == 0) throw std::runtime_error("layer planned for k_net_lds does not fit its LDS budget");
    if (nlds > 0) {
        na.u = u;
        na.so[0] = so0;
        na.so[1] = so1;
        na.params = P;
        na.aux = X;
        na.offs = E.p.dtab(c.dev_lds_offs);
        for (int n = 0; n < 2; n++) na.ci_off[n] = E.p.host_table[(size_t)c.dev_lds_offs + (size_t)n * na.offs_per_net];
        na.zero_bias = X + E.p.aux_zero;
        if (save != nullptr) {
            const LdsSave s = LdsSave::of(c.hc * c.wc, c.nk, c.gc, c.R);
            na.save = save;
            na.save_img = s.img;
            na.save_t1 = s.t1;
            na.save_t2 = s.t2;
            na.save_st = s.st;
        }
        if (nz != nullptr) {
            if (pend != nullptr || save != nullptr) throw std::logic_error("fused input noise: first inference layer only");
            na.nz = *nz;
        }
        if (pend != nullptr) {
            // buffer discipline of the deferred law (dry runs carry no real pointers): this layer's
            // input is the pending layer's output v_k, which must not be the u_k it is computed
            // from, and this layer's s/t outputs must not overwrite the pending s_pre / t it reads
            // (LDS layers alternate s/t sets by coupling index)
            if (!E.p.dry && (pend->v != u || pend->u == u || so0 == pend->s_pre || so0 == pend->t ||
                             so1 == pend->s_pre || so1 == pend->t))
                throw std::logic_error("deferred coupling: buffer aliasing (v_k / u_k / s,t sets)");
            na.pend = *pend;
            na.pend.comp = pend->mask_c == c.mask && pend->hc == c.hc && pend->wc == c.wc && pend->dc2 == c.dc1 ? 1 : 0;
        }
        const int ilds = (int)nlds;
        const double fl = 2.0 * B * net_flops(c);
        // algorithmic bytes: u1c in and s/t out per image and net, plus the per-element LN
        // gamma/beta (only the branch input windows of LN2) and the conv weights once per launch
        const double HWc = (double)c.hc * c.wc;
        int win = 0;
        for (int i = 0; i < na.nwin; i++) win += na.win_len[i];
        const double ln_floats = ln ? 2.0 * HWc * (c.R * (c.nk + win + c.gc) + c.nk) : 0.0;
        const double w_floats = net_flops(c) / (2.0 * HWc);
        const double by = 4.0 * (B * HWc * (c.dc1 + c.dc2) * 2 + 2 * (ln_floats + w_floats));
        E.record("k_net_lds", fl, by, [na, B, ilds](void* st) { launch_net_lds(na, B, ilds, (hipStream_t)st); });
    } else {
    if (nz != nullptr) throw std::logic_error("fused input noise: k_net_lds layers only");
    float* u1c = E.at<float>(L.u1c);
    // conv_in straight from u (k_pw tap mode: the mask gather inside the im2col loads) when packed
    const bool cin_tap = E.p.use_pw && c.net[0].ci_pw.size > 0;
    if (!cin_tap) {
        const float* uu = u;
        E.record("k_gather_u1c", 0, 4.0 * B * c.hc * c.wc * c.dc1 * 2,
                 [=](void* st) { launch_gather_u1c(uu, u1c, B, c.H, c.W, c.D, c.mask, c.hc, c.wc, c.dc1, (hipStream_t)st); });
    }
    float* y[2] = {E.at<float>(L.y[0]), E.at<float>(L.y[1])};
    float* t1[2] = {E.at<float>(L.t1[0]), E.at<float>(L.t1[1])};
    float* t2[2] = {E.at<float>(L.t2[0]), E.at<float>(L.t2[1])};
    float* so[2] = {E.at<float>(L.so[0]), E.at<float>(L.so[1])};
    // training forward with saved activations (TrainLayout::StreamSave): y_r and t2_r live in per-block
    // slices of the save area (conv_b writes y_{r+1} next to its residual y_r instead of in place), conv_a
    // also stores the full t1_r, and every LN tensor's statistics are folded once into [B][2]
    if (ss != nullptr && c.t2_mapped) throw std::logic_error("training save: mapped t2 layout");
    const size_t npx = (size_t)c.hc * c.wc;
    auto SY = [&](int n, int r) { return E.at<float>(ss->y[n]) + (size_t)r * B * npx * c.nk; };
    auto ST1 = [&](int n, int r) { return E.at<float>(ss->t1[n]) + (size_t)r * B * npx * c.nk; };
    auto ST2 = [&](int n, int r) { return E.at<float>(ss->t2[n]) + (size_t)r * B * npx * c.gc; };
    auto SST = [&](int n, int i) { return E.at<float>(ss->st[n]) + (size_t)i * B * 2; };
    if (ss != nullptr) {
        for (int n = 0; n < 2; n++) {
            y[n] = SY(n, 0);
            t2[n] = ST2(n, 0);
        }
        so[0] = so0;   // (so_save: the save area's raw conv_out)
        so[1] = so1;
    }
    Slab sl[2][3];   // [net][y, t1, t2]
    for (int n = 0; n < 2; n++)
        for (int k = 0; k < 3; k++) {
            sl[n][k].part = E.at<float>(L.st_part[n][k]);
        }
    // a producing launch reports the partial slots it wrote per image (set_parts); in_slab hands
    // that count on to the consumer
    auto out_slab = [&](int n, int k, int) { return ln ? sl[n][k] : Slab{}; };
    // more slots than a consumer wave fetches in its prologue (64 x LN_FETCH = 512: the 128x128 layers):
    // merged once per image by k_ln_merge instead of by every consumer workgroup for each of its images
    // (the 64x64 layers' slots are folded by the consumers: 70 fewer launches per cfg4 step)
#ifdef CNF_DIAG_NO_LN_MERGE   // (diagnostic builds: the consumers fold every slot)
    constexpr int ln_merge_over = 1 << 30;
#else
    constexpr int ln_merge_over = 64 * LN_FETCH;
#endif
    auto set_parts = [&](int k, int nparts) {
        if (ln && nparts > ln_merge_over) {
            float* p0 = sl[0][k].part;
            float* p1 = sl[1][k].part;
            const int np = nparts, ps = L.st_parts;
            E.record("k_ln_merge", 0, 16.0 * B * np * 2 + 32.0 * B,
                     [=](void* st) { launch_ln_merge(p0, p1, np, ps, B, (hipStream_t)st); });
            nparts = 1;
        }
        for (int n = 0; n < 2; n++) sl[n][k].nparts = nparts;
    };
    // training save: the statistics of LN tensor i (see TrainLayout::StreamSave) from slab k's slots, folded
    // by one k_ln_final per residual block (flush_stats before conv_b overwrites slab 0, and at the end):
    // the three slabs hold y_r, t1_r and t2_r until then
    LnFinalSet pend_stats{};
    pend_stats.part_stride = L.st_parts;
    auto flush_stats = [&]() {
        if (pend_stats.count == 0) return;
        const LnFinalSet fs = pend_stats;
        double bytes = 0.0;
        for (int q = 0; q < fs.count; q++) bytes += 16.0 * B * fs.nparts[q] * 2;
        E.record("k_ln_final", 0, bytes, [=](void* st) { launch_ln_final(fs, B, (hipStream_t)st); });
        pend_stats.count = 0;
    };
    auto save_stats = [&](int k, int i) {
        if (ss == nullptr || !ln) return;
        if (pend_stats.count == LNF_MAX) flush_stats();
        const int q = pend_stats.count++;
        pend_stats.part[q][0] = sl[0][k].part;
        pend_stats.part[q][1] = sl[1][k].part;
        pend_stats.st[q][0] = SST(0, i);
        pend_stats.st[q][1] = SST(1, i);
        pend_stats.nparts[q] = sl[0][k].nparts;
    };
    auto in_slab = [&](int n, int k) { return ln ? sl[n][k] : Slab{}; };
    const float* none = nullptr;
    // LN2 gamma/beta in t1's layout: the aux copies gathered to the compact layout, or the parameters
    auto ln2g = [&](const RBParams& rb) { return c.t1_compact ? X + rb.ln2c_g : P + rb.ln2g; };
    auto ln2b = [&](const RBParams& rb) { return c.t1_compact ? X + rb.ln2c_b : P + rb.ln2b; };
    auto ln3g = [&](const RBParams& rb) { return c.t2_mapped ? X + rb.ln3c_g : P + rb.ln3g; };
    auto ln3b = [&](const RBParams& rb) { return c.t2_mapped ? X + rb.ln3c_b : P + rb.ln3b; };
    // device-table maps of the mapped layouts (fake, never dereferenced, in dry runs)
    auto dmap = [&](int off) -> const int* {
        return E.p.dtab(off);
    };

    // conv_in (:1114-1119 / :1159-1164): u1c -> y, both nets in one launch
    if (cin_tap) {
        std::vector<ProbSpec> pr;
        for (int n = 0; n < 2; n++) {
            const NetParams& np = c.net[n];
            pr.push_back(ProbSpec{u, 9 * c.dc1, 0, 9 * c.dc1, Slab{}, none, none, 0, X + np.ci_pw.w, X + np.ci_pw.b,
                                  y[n], c.nk, 0, c.nk, none, out_slab(n, 0, 4 * nt1), 0, 1});
        }
        const TapSrc ts{c.mask, c.W, c.D, c.dc1, c.H * c.W * c.D};
        set_parts(0, conv_launch(E, 1, ROLE_CONV_IN, c.hc, c.wc, pr, ~0ull, &ts));
    } else {
        std::vector<ProbSpec> pr;
        for (int n = 0; n < 2; n++) {
            const NetParams& np = c.net[n];
            pr.push_back(ProbSpec{u1c, c.dc1, 0, c.dc1, Slab{}, none, none, 0, X + np.ci.w, X + np.ci.b, y[n], c.nk, 0,
                                  c.nk, none, out_slab(n, 0, 4 * nt3), 0, 1});
        }
        set_parts(0, conv_launch(E, 3, ROLE_CONV_IN, c.hc, c.wc, pr));
    }
    save_stats(0, 0);
    for (int r = 0; r < c.R; r++) {
        if (ss != nullptr)
            for (int n = 0; n < 2; n++) t2[n] = ST2(n, r);
        // conv_a: LN1(LReLU(y)) -> 1x1 -> t1
        {
            std::vector<ProbSpec> pr;
            for (int n = 0; n < 2; n++) {
                const RBParams& rb = c.net[n].rb[r];
                pr.push_back(ProbSpec{y[n], c.nk, 0, c.nk, in_slab(n, 0), ln ? P + rb.ln1g : none,
                                      ln ? P + rb.ln1b : none, 1, X + rb.ca.w, X + rb.ca.b, t1[n], c.t1_cs, 0, c.nk,
                                      none, out_slab(n, 1, 4 * nt1), 0, 1});
                // training: the full t1_r for the backward's LN2 from the same launch (k_pw's second
                // store; its dual-store instantiations exist for LN on only -- without LN the separate
                // launch below writes it)
                if (ss != nullptr && ln) pr.back().out2 = ST1(n, r);
            }
            // only the channels the branches read are stored (into their consumers' sub-tensors when
            // t1_compact); the LN2 statistics still cover all nk channels
            const int* t1map = c.t1_compact ? E.p.dtab(c.dev_t1_map) : nullptr;
            bool dual = false;
            set_parts(1, conv_launch(E, 1, ROLE_CONV_A, c.hc, c.wc, pr, c.t1_used, nullptr, t1map, nullptr, &dual));
            dual = dual && ln;   // (out2 is set with LN only: without it k_pw made no second store)
            if (ss != nullptr && dual) save_stats(1, c.R + 1 + r);
            if (ss != nullptr && !dual) {
                // the full t1_r for the backward's LN2 (the compact t1 above holds only the branch windows)
                std::vector<ProbSpec> pf;
                for (int n = 0; n < 2; n++) {
                    const RBParams& rb = c.net[n].rb[r];
                    pf.push_back(ProbSpec{y[n], c.nk, 0, c.nk, in_slab(n, 0), ln ? P + rb.ln1g : none,
                                          ln ? P + rb.ln1b : none, 1, X + rb.ca.w, X + rb.ca.b, ST1(n, r), c.nk, 0, c.nk,
                                          none, Slab{}, 0, 1});
                }
                conv_launch(E, 1, ROLE_CONV_A, c.hc, c.wc, pf);
                save_stats(1, c.R + 1 + r);
            }
        }
        // grouped dilated branches: LN2(LReLU(t1)) -> 3x3 dil d -> t2[:, out_off:out_off+cout]. The k_gc
        // launch (when planned) takes its branches first; every other branch runs as a k_pw tap-mode
        // launch over its im2col row when that row fits (9 cin <= 128), the rest as one k_conv<3>.
        // Each launch's LN3 partial slots follow the previous ones'.
        int base = 0;
        std::vector<char> done(nbr, 0);
        for (const Coupling::GcGroup& gg : c.gcg) {
            const int ng = (int)gg.br.size();
            GcArgs ga;
            std::memset(&ga, 0, sizeof(ga));
            for (int n = 0; n < 2; n++) {
                const RBParams& rb = c.net[n].rb[r];
                ga.in[n] = t1[n];
                ga.out[n] = t2[n];
                ga.in_part[n] = ln ? sl[n][1].part : nullptr;
                ga.out_part[n] = ln ? sl[n][2].part + (size_t)base * LNP : nullptr;   // after earlier launches' slots
                ga.gamma[n] = ln ? ln2g(rb) : nullptr;
                ga.beta[n] = ln ? ln2b(rb) : nullptr;
                for (int k = 0; k < ng; k++) {
                    ga.w[n][k] = X + rb.gc[gg.br[k]].w;
                    ga.b[n][k] = X + rb.gc[gg.br[k]].b;
                }
            }
            for (int k = 0; k < ng; k++) {
                ga.s.br[k] = gg.gcb[k];
                done[gg.br[k]] = 1;
            }
            ga.s.nbr = ng;
            ga.s.H = c.hc;
            ga.s.W = c.wc;
            ga.s.in_cs = c.t1_cs;
            ga.s.out_cs = c.t2_cs;
            ga.B = B;
            ga.s.TH = gg.TH;
            ga.s.TW = gg.TW;
            ga.s.tiles_x = gg.tiles_x;
            ga.s.tiles_per_img = gg.tiles();
            ga.s.ps = gg.ps;
            ga.s.nbk = gg.nbk;
            ga.s.tpp = gg.tpp;
            ga.s.nw = gg.nw;
            ga.s.pd = gg.pd;
            ga.in_nparts = sl[0][1].nparts;
            ga.part_stride = L.st_parts;
            // images per workgroup: one workgroup per CU, looping over its images with the next
            // image's band staged behind the current one's MFMAs
            // (16 / nw workgroups per CU)
            const int64_t units = (int64_t)ga.s.tiles_per_img * 2 * B;
            const int64_t slots = 256LL * gc_wg_per_cu(gg.nw);
            ga.ipw = (int)std::min<int64_t>(16, std::max<int64_t>(1, (units + slots - 1) / slots));
#ifdef CNF_DIAG
            if (const char* e = std::getenv("CNF_GC_IPW")) ga.ipw = std::atoi(e);   // diagnostics
#endif
            ga.s.band_bytes = gg.band_bytes;
            ga.s.lnst = (ga.in_part[0] ? 1 : 0) | (ga.out_part[0] ? 2 : 0);
            const int gcw = gc_waves(ga);
            if (base + gcw * ga.s.tiles_per_img > L.st_parts) throw std::runtime_error("k_gc: LN partial slab too small");
            const int grid_x = ga.s.tiles_per_img * ((B + ga.ipw - 1) / ga.ipw);
            const int ilds = gg.lds;
            double fl = 0, by = 0;
            int win = 0;
            for (int k = 0; k < ng; k++) {
                const Branch& b = c.br[gg.br[k]];
                fl += 2.0 * B * c.hc * c.wc * 9.0 * b.cin * b.cout * 2;
                win += b.cin;
                by += 4.0 * B * c.hc * c.wc * b.cout * 2;
            }
            by += 4.0 * B * c.hc * c.wc * win * 2 + (ln ? 4.0 * 2 * c.hc * c.wc * win * 2 : 0.0);
            if (E.p.dry) {
                bool seen = false;
                for (const GcShape& o : E.p.gc_launch) seen = seen || std::memcmp(&o, &ga.s, sizeof(GcShape)) == 0;
                if (!seen) E.p.gc_launch.push_back(ga.s);
            }
            E.record("k_gc", fl, by, [ga, grid_x, ilds](void* st) { launch_gc(ga, grid_x, ilds, (hipStream_t)st); });
            base += gcw * ga.s.tiles_per_img;   // one slot per k_gc wave
        }
        {
            std::vector<ProbSpec> pr;
            for (int bi = 0; bi < nbr; bi++) {
                const Branch& b = c.br[bi];
                if (done[bi] || !(E.p.use_pw && c.net[0].rb[r].gpw[bi].size > 0)) continue;
                std::vector<ProbSpec> pt;
                for (int n = 0; n < 2; n++) {
                    const RBParams& rb = c.net[n].rb[r];
                    pt.push_back(ProbSpec{t1[n], 9 * b.cin, 0, 9 * b.cin, in_slab(n, 1), ln ? ln2g(rb) : none,
                                          ln ? ln2b(rb) : none, 1, X + rb.gpw[bi].w, X + rb.gpw[bi].b, t2[n], c.t2_cs,
                                          b.out_off, b.cout, none, out_slab(n, 2, 0), base, 1});
                }
                const int* bmap = c.t2_mapped ? dmap(c.dev_t2_bmap[bi]) : nullptr;
                TapSrc ts{-1, c.wc, c.t1_pcs[bi], b.cin, c.hc * c.wc * c.t1_cs};
                ts.dil = b.dil;
                ts.off = c.t1_off[bi];
                base += conv_launch(E, 1, ROLE_GC, c.hc, c.wc, pt, ~0ull, &ts, bmap);
                done[bi] = 1;
            }
            int nrest = 0;
            for (int n = 0; n < 2; n++) {
                const RBParams& rb = c.net[n].rb[r];
                int k = 0;
                for (int bi = 0; bi < nbr; bi++) {
                    const Branch& b = c.br[bi];
                    if (done[bi]) continue;
                    if (c.t1_compact || c.t2_mapped) throw std::logic_error("k_conv<3> branch on a mapped t1 / t2 layout");
                    pr.push_back(ProbSpec{t1[n], c.nk, b.cin_off, b.cin, in_slab(n, 1), ln ? ln2g(rb) : none,
                                          ln ? ln2b(rb) : none, 1, X + rb.gc[bi].w, X + rb.gc[bi].b, t2[n], c.gc,
                                          b.out_off, b.cout, none, out_slab(n, 2, 0), base + k * nt3 * 4, b.dil});
                    k++;
                }
                nrest = k;
            }
            if (!pr.empty()) {
                base += nrest * conv_launch(E, 3, ROLE_GC, c.hc, c.wc, pr);
            }
            if (base > L.st_parts) throw std::runtime_error("grouped branches: LN partial slab too small");
            set_parts(2, base);
            save_stats(2, 2 * c.R + 1 + r);
        }
        // conv_b: LN3(LReLU(t2)) -> 1x1 -> + shortcut -> y (in place)
        {
            flush_stats();   // (conv_b writes slab 0's slots: y_r's statistics first)
            std::vector<ProbSpec> pr;
            for (int n = 0; n < 2; n++) {
                const RBParams& rb = c.net[n].rb[r];
                pr.push_back(ProbSpec{t2[n], c.t2_cs, 0, c.gc, in_slab(n, 2), ln ? ln3g(rb) : none,
                                      ln ? ln3b(rb) : none, 1, X + rb.cb.w, X + rb.cb.b,
                                      ss != nullptr ? SY(n, r + 1) : y[n], c.nk, 0, c.nk, y[n],
                                      out_slab(n, 0, 4 * nt1), 0, 1});
            }
            set_parts(0, conv_launch(E, 1, ROLE_CONV_B, c.hc, c.wc, pr, ~0ull, nullptr, nullptr,
                                     c.t2_mapped ? dmap(c.dev_t2_qmap) : nullptr));
            if (ss != nullptr)
                for (int n = 0; n < 2; n++) y[n] = SY(n, r + 1);
            save_stats(0, r + 1);
        }
    }
    flush_stats();
    // conv_out: LN_out(LReLU(y)) -> 3x3 -> so (raw A pre-tanh / b); > 64 outputs in 64-channel chunks
    {
        std::vector<ProbSpec> pr;
        for (int n = 0; n < 2; n++) {
            const NetParams& np = c.net[n];
            if (!np.co_chunks.empty()) {
                for (size_t k = 0; k < np.co_chunks.size(); k++)
                    pr.push_back(ProbSpec{y[n], c.nk, 0, c.nk, in_slab(n, 0), ln ? P + np.ln_out_g : none,
                                          ln ? P + np.ln_out_b : none, 1, X + np.co_chunks[k].w,
                                          X + np.co_chunks[k].b, so[n], c.dc2, (int)(64 * k),
                                          np.co_chunks[k].cout, none, Slab{}, 0, 1});
                continue;
            }
            pr.push_back(ProbSpec{y[n], c.nk, 0, c.nk, in_slab(n, 0), ln ? P + np.ln_out_g : none,
                                  ln ? P + np.ln_out_b : none, 1, X + np.co.w, X + np.co.b, so[n], c.dc2, 0, c.dc2,
                                  none, Slab{}, 0, 1});
        }
        if (c.net[0].co.fmt == PK_TAP && E.p.tap_pw && 9 * c.dc2 <= c.nk && pr.size() == 2) {
            // tap GEMM C = LN_out(LReLU(y)) . W_tap as a streamed 1x1 conv into the dead t1 buffer;
            // k_coupling finishes the 3x3 (tap sums + bias) where it reads s and t
            for (int n = 0; n < 2; n++) {
                ProbSpec& q = pr[n];
                q.bias = X + E.p.aux_zero;
                q.out = t1[n];
                q.out_cs = q.cout = 9 * c.dc2;
                q.out_off = 0;
                tap_c[n] = t1[n];
                tap_b[n] = X + c.net[n].co.b;
            }
            conv_launch(E, 1, ROLE_CONV_OUT, c.hc, c.wc, pr);
        } else if (c.net[0].co.fmt == PK_TAP) {
            convtap_launch(E, c.hc, c.wc, pr);
        } else {
            conv_launch(E, 3, ROLE_CONV_OUT, c.hc, c.wc, pr);
        }
    }
    }  // streamed path
    // affine coupling law + decompress + log-det partials
    if (defer) {
        CoupPend& q = *out_pend;
        q = CoupPend{};
        q.u = u;
        q.s_pre = so0;
        q.t = so1;
        q.tanh_w = P + c.net[0].tanh_w;
        q.v = v;
        q.ld_part = ld_part;
        q.mask_c = c.mask_c;
        q.hc = c.hc;
        q.wc = c.wc;
        q.dc2 = c.dc2;
        q.np = E.L.ld_parts;
        q.on = 1;
        q.mask = c.mask;
        q.dc1 = c.dc1;
        q.W = c.W;
        q.D = c.D;
        q.dir = dir;
        return;
    }
    {
        CoupArgs ca;
        ca.u = u;
        ca.v = v;
        ca.s_pre = so0;
        ca.t = so1;
        ca.tanh_w = P + c.net[0].tanh_w;
        ca.ld_part = ld_part;
        ca.H = c.H;
        ca.W = c.W;
        ca.D = c.D;
        ca.mask = c.mask;
        ca.mask_c = c.mask_c;
        ca.hc = c.hc;
        ca.wc = c.wc;
        ca.dc1 = c.dc1;
        ca.dc2 = c.dc2;
        ca.dir = dir;
        for (int n = 0; n < 2; n++) {
            ca.tc[n] = tap_c[n];
            ca.tbias[n] = tap_b[n];
            ca.so_w[n] = n == 0 ? so0 : so1;
        }
        const int np = E.L.ld_parts;
        E.record("k_coupling", 0, 4.0 * B * c.H * c.W * c.D * 2 + 8.0 * B * c.hc * c.wc * c.dc2,
                 [ca, B, np](void* st) { launch_coupling(ca, B, np, (hipStream_t)st); });
    }
}

static void ensure_tables(Plan& p) {
    int dev = 0;
    hip_check(hipGetDevice(&dev), "hipGetDevice");
    if (p.dev_table != nullptr && p.device == dev) return;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    // uploading is not capturable: the first call on a device must run eagerly
    if (hipStreamIsCapturing(nullptr, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone)
        throw std::runtime_error("plan tables not uploaded yet (call cnf_pack_params before graph capture)");
    // NLL_SLOTS ints past the table: cnf_nll's completion counters (zero between launches)
    size_t nb = (p.host_table.size() + Plan::NLL_SLOTS) * sizeof(int);
    hip_check(hipMalloc(&p.dev_table, nb), "hipMalloc(table)");
    hip_check(hipMemset(p.dev_table, 0, nb), "hipMemset(table)");
    if (!p.host_table.empty())
        hip_check(hipMemcpy(p.dev_table, p.host_table.data(), p.host_table.size() * sizeof(int), hipMemcpyHostToDevice),
                  "hipMemcpy(table)");
    size_t na = std::max<size_t>(1, p.aux_map.size()) * sizeof(int64_t);
    hip_check(hipMalloc(&p.dev_aux_map, na), "hipMalloc(aux map)");
    if (!p.aux_map.empty())
        hip_check(hipMemcpy(p.dev_aux_map, p.aux_map.data(), p.aux_map.size() * sizeof(int64_t), hipMemcpyHostToDevice),
                  "hipMemcpy(aux map)");
    size_t nbw = std::max<size_t>(1, p.bw_map.size()) * sizeof(int64_t);
    hip_check(hipMalloc(&p.dev_bw_map, nbw), "hipMalloc(bw map)");
    if (!p.bw_map.empty())
        hip_check(hipMemcpy(p.dev_bw_map, p.bw_map.data(), p.bw_map.size() * sizeof(int64_t), hipMemcpyHostToDevice),
                  "hipMemcpy(bw map)");
    p.device = dev;
}

static void check_launch() { hip_check(hipGetLastError(), "kernel launch"); }

}  // namespace cnf

using namespace cnf;

// ================================================================================================
// C ABI
// ================================================================================================
extern "C" {

const char* cnf_last_error(void) { return g_err.c_str(); }
const char* cnf_version(void) { return "cnf-mi355x 0.1 (gfx950)"; }

int cnf_plan_create(const cnf_flow_desc* desc, cnf_plan** out) {
    if (!out) return fail(CNF_E_INVALID, "null out");
    *out = nullptr;
    CNF_TRY
    Plan* p = build_plan(desc);   // (parses desc->debug_options into p->opts)
    OptScope os(&p->opts);
    p->use_pw = p->tap_pw = p->opts.pw != 0;
    // validate tiling / LDS budget for every layer up-front
    for (const auto& c : p->couplings) (void)conv_geo(c.hc, c.wc);
    // training: k_net_lds layers whose fused backward fits LDS use it (debug option LDS_BWD=0: none)
    const bool lds_bwd = p->opts.lds_bwd != 0;
    for (auto& c : p->couplings) {
        LdsBwdArgs a;
        c.lds_bwd = lds_bwd && c.use_lds && ldsbwd_setup(*p, c, a) > 0;
    }
    *out = new cnf_plan{p};
    return CNF_OK;
    CNF_CATCH
}

void cnf_plan_destroy(cnf_plan* plan) {
    if (!plan) return;
    if (plan->p) {
        if (plan->p->dev_table) (void)hipFree(plan->p->dev_table);
        if (plan->p->dev_aux_map) (void)hipFree(plan->p->dev_aux_map);
        if (plan->p->dev_bw_map) (void)hipFree(plan->p->dev_bw_map);
        for (hipEvent_t e : plan->p->ev) (void)hipEventDestroy(e);
        if (plan->p->ev_fork) (void)hipEventDestroy(plan->p->ev_fork);
        if (plan->p->ev_join) (void)hipEventDestroy(plan->p->ev_join);
        if (plan->p->side) (void)hipStreamDestroy(plan->p->side);
        for (hipStream_t s : plan->p->wside)
            if (s) (void)hipStreamDestroy(s);
        for (hipEvent_t e : plan->p->tev) (void)hipEventDestroy(e);
        for (hipEvent_t e : plan->p->nll_ev)
            if (e) (void)hipEventDestroy(e);
        delete plan->p;
    }
    delete plan;
}

int cnf_plan_num_layers(const cnf_plan* plan) { return plan ? (int)plan->p->layers.size() : -1; }

int cnf_plan_layer_info(const cnf_plan* plan, int layer, cnf_layer_info* out) {
    OptScope os_(plan ? &plan->p->opts : nullptr);
    if (!plan || !out) return fail(CNF_E_INVALID, "null argument");
    const Plan& p = *plan->p;
    if (layer < 0 || layer >= (int)p.layers.size()) return fail(CNF_E_INVALID, "layer index out of range");
    std::memset(out, 0, sizeof(*out));
    const Layer& L = p.layers[layer];
    out->kind = L.kind;
    out->coupling_index = L.ci;
    out->block = L.block;
    out->h = L.h;
    out->w = L.w;
    out->d = L.d;
    out->num_prev_factors = L.npf;
    if (L.kind == CNF_LAYER_COUPLING) {
        out->fused_net = p.couplings[L.ci].use_lds ? 1 : 0;
        const Coupling& c = p.couplings[L.ci];
        out->mask = c.mask;
        out->hc = c.hc;
        out->wc = c.wc;
        out->dc1 = c.dc1;
        out->dc2 = c.dc2;
        out->num_kernels = c.nk;
        out->cardinality = c.card;
        out->num_res_blocks = c.R;
        out->num_dilations = (int)c.dils.size();
        for (int i = 0; i < (int)c.dils.size() && i < 8; i++) out->dilations[i] = c.dils[i];
    }
    return CNF_OK;
}

int64_t cnf_plan_num_params(const cnf_plan* plan) { return plan ? plan->p->n_params : -1; }
int cnf_plan_num_param_tensors(const cnf_plan* plan) { return plan ? (int)plan->p->params.size() : -1; }

int cnf_plan_param_tensor(const cnf_plan* plan, int index, char* name, int name_cap, int64_t* offset, int* ndim,
                          int shape[4]) {
    OptScope os_(plan ? &plan->p->opts : nullptr);
    if (!plan) return fail(CNF_E_INVALID, "null plan");
    const Plan& p = *plan->p;
    if (index < 0 || index >= (int)p.params.size()) return fail(CNF_E_INVALID, "param index out of range");
    const ParamTensor& t = p.params[index];
    if (name && name_cap > 0) {
        std::snprintf(name, (size_t)name_cap, "%s", t.name.c_str());
    }
    if (offset) *offset = t.offset;
    if (ndim) *ndim = (int)t.shape.size();
    if (shape)
        for (int i = 0; i < 4; i++) shape[i] = i < (int)t.shape.size() ? t.shape[i] : 0;
    return CNF_OK;
}

int64_t cnf_plan_aux_floats(const cnf_plan* plan) { return plan ? std::max<int64_t>(1, plan->p->n_aux) : -1; }

int cnf_pack_params(cnf_plan* plan, const float* params, float* aux, void* stream) {
    OptScope os_(plan ? &plan->p->opts : nullptr);
    if (!plan || !params || !aux) return fail(CNF_E_INVALID, "null argument");
    CNF_TRY
    Plan& p = *plan->p;
    ensure_tables(p);
    if (p.n_aux > 0) launch_pack(params, p.dev_aux_map, aux, (long long)p.n_aux, (hipStream_t)stream);
    check_launch();
    return CNF_OK;
    CNF_CATCH
}

size_t cnf_plan_workspace_bytes(const cnf_plan* plan, int B) {
    OptScope os_(plan ? &plan->p->opts : nullptr);
    if (!plan || B <= 0) return 0;
    return plan->p->layout(B).total;
}

}  // extern "C"

// the forward schedule; save_inputs: also copy every coupling layer's input into the training
// workspace (cnf_flow_forward_train)
// nz (cnf_flow_forward_noise): xy is the caller's buffer for the noisy input, which the first coupling's
// k_net_lds writes while gathering from nz->src with the noise applied (a k_noise pass into it first when
// that layer is streamed)
static void flow_forward(Plan& p, const float* params, const float* aux, const float* xy, float* zy,
                         float* logdet_per_image, void* workspace, int B, hipStream_t stream, bool save_inputs,
                         const InputPrepArgs* nz = nullptr) {
    if (!p.dry) ensure_tables(p);
    p.recorded.clear();
    Exec E{p, params, aux, (char*)workspace, p.layout(B), B, stream};
    TrainLayout TL;
    if (save_inputs) TL = p.train_layout(B);
    const WsLayout& L = E.L;
    double* ld = E.at<double>(L.ld);
    float* buf[2] = {E.at<float>(L.uv[0]), E.at<float>(L.uv[1])};
    const float* cur = xy;
    int which = 0;
    size_t bi = 0;
    const int nuv = (int)L.n_uv;
    const bool nz_fused = nz != nullptr && !save_inputs && !p.layers.empty() &&
                          p.layers[0].kind == CNF_LAYER_COUPLING && p.couplings[p.layers[0].ci].use_lds;
    if (nz != nullptr && !nz_fused) {
        const InputPrepArgs q = *nz;
        float* dst = const_cast<float*>(xy);
        const long long n = (long long)B * p.desc.io_h * p.desc.io_w * p.desc.io_d;
        E.record("k_prep", 0, 8.0 * n, [=](void* st) { launch_input_prep(dst, n, q, (hipStream_t)st); });
    }
    // a k_net_lds layer followed directly by another one leaves its coupling law to that layer's
    // kernel (CoupPend): no k_coupling launch for it. Not when saving layer inputs (training).
    const bool fuse = p.opts.fuse_coupling != 0;   // (debug option FUSE_COUPLING=0: a k_coupling per layer)
    CoupPend pend;
    bool have_pend = false;
    // training: a layer whose output is the next coupling's input writes it straight into that coupling's
    // save slot (no copy of every layer input; only the first coupling's, which reads xy)
    auto save_slot_after = [&](size_t li) -> float* {
        size_t nx = li + 1;
        while (nx < p.layers.size() && p.layers[nx].kind == CNF_LAYER_SQUEEZE) nx++;
        if (!save_inputs || nx >= p.layers.size() || p.layers[nx].kind != CNF_LAYER_COUPLING) return nullptr;
        return E.at<float>(TL.save_u[p.couplings[p.layers[nx].ci].index]);
    };
    for (size_t li = 0; li < p.layers.size(); li++) {
        const Layer& ly = p.layers[li];
        if (ly.kind == CNF_LAYER_COUPLING) {
            const Coupling& c = p.couplings[ly.ci];
            // the next layer that launches anything (squeezes are folded into the factor maps)
            size_t nx = li + 1;
            while (nx < p.layers.size() && p.layers[nx].kind == CNF_LAYER_SQUEEZE) nx++;
            const bool next_lds = nx < p.layers.size() && p.layers[nx].kind == CNF_LAYER_COUPLING &&
                                  p.couplings[p.layers[nx].ci].use_lds;
            const bool next_maps = nx >= p.layers.size() || p.layers[nx].kind == CNF_LAYER_FACTOR;
            const bool defer = fuse && !save_inputs && c.use_lds && (next_lds || next_maps);
            float* nxt = buf[which];
            if (float* slot = save_slot_after(li)) nxt = slot;
            if (save_inputs && cur != E.at<float>(TL.save_u[c.index])) {
                float* dst = E.at<float>(TL.save_u[c.index]);
                const float* src = cur;
                const size_t bytes = (size_t)B * c.H * c.W * c.D * 4;
                E.record("copy", 0, 2.0 * bytes, [=](void* st) {
                    (void)hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)st);
                });
            }
            CoupPend next;
            float* save = nullptr;
            float* so_save[2] = {nullptr, nullptr};
            if (save_inputs && c.lds_bwd) {   // the fused LDS backward's activations
                save = E.at<float>(TL.act_save[c.index]);
                so_save[0] = E.at<float>(TL.so_save[c.index]);
                so_save[1] = so_save[0] + (size_t)B * c.hc * c.wc * c.dc2;
            }
            const TrainLayout::StreamSave* ss =
                save_inputs && !c.use_lds && TL.has_ssave[c.index] ? &TL.ssave[c.index] : nullptr;
            if (ss != nullptr) {   // the raw conv_out (k_coupling's so_w in tap mode) into the save area
                so_save[0] = E.at<float>(ss->so);
                so_save[1] = so_save[0] + (size_t)B * c.hc * c.wc * c.dc2;
            }
            run_coupling(E, c, cur, nxt, ld + (size_t)c.index * B * L.ld_parts, +1, have_pend ? &pend : nullptr,
                         defer, &next, save, (save || ss) ? so_save : nullptr, ss, nz_fused && li == 0 ? nz : nullptr);
            pend = next;
            have_pend = defer;
            cur = nxt;
            which ^= 1;
        } else if (ly.kind == CNF_LAYER_FACTOR) {
            // squeeze (:179) + factor (:276-286) at a block boundary: kept half -> next buffer,
            // factored half -> its final xy-layout position in zy (:1762-1770 restoration).
            const Boundary& b = p.boundaries[bi++];
            // with a pending coupling the maps read u_k (the other buffer) on the fly, and v_k's
            // own buffer (cur, never written) takes the kept half
            float* nxt = have_pend ? const_cast<float*>(cur) : buf[which];
            if (!have_pend)
                if (float* slot = save_slot_after(li)) nxt = slot;
            const bool flip = !have_pend;
            const int* T = p.dtab(0);
            const float* src = cur;
            const int ncur = b.n_cur, nnext = b.n_next, nfac = b.n_fac;
            const int* ks = T + b.dev_keep_src;
            const int* fs = T + b.dev_fac_src;
            const int* fo = T + b.dev_fac_orig;
            // keep gather -> next buffer and factored scatter -> zy: one launch (reading v of a
            // pending coupling on the fly, with that layer's log-det partials)
            MapOp mk, mf;
            mk.src = src, mk.dst = nxt, mk.sidx = ks, mk.n = nnext, mk.ss = ncur, mk.ds = nnext;
            mf.src = src, mf.dst = zy, mf.sidx = fs, mf.didx = fo, mf.n = nfac, mf.ss = ncur, mf.ds = nuv;
            const CoupPend q = have_pend ? pend : CoupPend{};
            mk.pend = mf.pend = q.on;
            if (!p.dry && q.on && (nxt == q.u || zy == q.u)) throw std::logic_error("k_map2 would overwrite the u_k it reads");
            have_pend = false;
            E.record("k_map2", 0, 8.0 * B * (nnext + nfac),
                     [=](void* st) { launch_map2(mk, mf, LdReduce{}, q, B, (hipStream_t)st); });
            cur = nxt;
            if (flip) which ^= 1;
        }
    }
    {
        // final scatter (restore to xy's layout) and the per-image log-det reduction: one launch
        MapOp mf;
        mf.src = cur, mf.dst = zy, mf.didx = p.dtab(p.dev_final_orig), mf.n = p.last_n, mf.ss = p.last_n;
        mf.ds = nuv;
        LdReduce r;
        r.part = ld, r.out = logdet_per_image, r.nl = (int)p.couplings.size(), r.np = L.ld_parts, r.accumulate = 0;
        const CoupPend q = have_pend ? pend : CoupPend{};
        mf.pend = q.on;
        if (have_pend) r.nl -= 1;   // the pending layer is the last one: its log-det sum goes straight into the total
        E.record("k_map2", 0, 8.0 * B * p.last_n, [=](void* st) { launch_map2(mf, MapOp{}, r, q, B, (hipStream_t)st); });
    }
    if (!p.dry) check_launch();
}

extern "C" {

int cnf_flow_forward(cnf_plan* plan, const float* params, const float* aux, const float* xy, float* zy,
                     float* logdet_per_image, void* workspace, int B, void* stream) {
    OptScope os_(plan ? &plan->p->opts : nullptr);
    if (!plan || !params || !aux || !xy || !zy || !logdet_per_image || !workspace || B <= 0)
        return fail(CNF_E_INVALID, "null argument or B <= 0");
    if (xy == zy) return fail(CNF_E_INVALID, "xy and zy must not alias (out-of-place only)");
    CNF_TRY
    flow_forward(*plan->p, params, aux, xy, zy, logdet_per_image, workspace, B, (hipStream_t)stream, false);
    return CNF_OK;
    CNF_CATCH
}

int cnf_flow_forward_noise(cnf_plan* plan, const float* params, const float* aux, const float* xy, float logit_a,
                           float alpha, uint64_t seed, uint64_t offset, float* xy_noisy, float* zy,
                           float* logdet_per_image, void* workspace, int B, void* stream) {
    OptScope os_(plan ? &plan->p->opts : nullptr);
    if (!plan || !params || !aux || !xy || !xy_noisy || !zy || !logdet_per_image || !workspace || B <= 0)
        return fail(CNF_E_INVALID, "null argument or B <= 0");
    if (xy == zy || xy_noisy == zy || xy_noisy == xy)
        return fail(CNF_E_INVALID, "xy, xy_noisy and zy must not alias (out-of-place only)");
    if (logit_a != 0.f && !(logit_a > 0.f && logit_a < 0.5f))
        return fail(CNF_E_INVALID, "logit_a must be 0 (no logit map) or in (0, 0.5)");
    CNF_TRY
    InputPrepArgs nz;
    std::memset(&nz, 0, sizeof(nz));
    nz.src = xy;
    nz.alpha = alpha;
    nz.seed = seed;
    nz.off = offset;
    nz.logit = logit_a != 0.f ? 1 : 0;
    nz.x_d = plan->p->desc.x_d;
    nz.D = plan->p->desc.io_d;
    if (nz.logit) nz.lk = logit_consts(logit_a);
    flow_forward(*plan->p, params, aux, xy_noisy, zy, logdet_per_image, workspace, B, (hipStream_t)stream, false, &nz);
    return CNF_OK;
    CNF_CATCH
}

size_t cnf_plan_train_workspace_bytes(const cnf_plan* plan, int B) {
    OptScope os_(plan ? &plan->p->opts : nullptr);
    if (!plan || B <= 0) return 0;
    try {
        return plan->p->train_layout(B).total;
    } catch (...) {
        return 0;
    }
}

int cnf_flow_forward_train(cnf_plan* plan, const float* params, const float* aux, const float* xy, float* zy,
                           float* logdet_per_image, void* train_workspace, int B, void* stream) {
    OptScope os_(plan ? &plan->p->opts : nullptr);
    if (!plan || !params || !aux || !xy || !zy || !logdet_per_image || !train_workspace || B <= 0)
        return fail(CNF_E_INVALID, "null argument or B <= 0");
    if (xy == zy) return fail(CNF_E_INVALID, "xy and zy must not alias (out-of-place only)");
    CNF_TRY
    flow_forward(*plan->p, params, aux, xy, zy, logdet_per_image, train_workspace, B, (hipStream_t)stream, true);
    return CNF_OK;
    CNF_CATCH
}

int cnf_flow_backward(cnf_plan* plan, const float* params, const float* xy, const float* zy, void* train_workspace,
                      int B, float inv_batch, float* dparams, void* stream) {
    OptScope os_(plan ? &plan->p->opts : nullptr);
    if (!plan || !params || !xy || !zy || !train_workspace || !dparams || B <= 0)
        return fail(CNF_E_INVALID, "null argument or B <= 0");
    CNF_TRY
    Plan& p = *plan->p;
    ensure_tables(p);
    flow_backward(p, params, xy, zy, train_workspace, B, inv_batch, dparams, (hipStream_t)stream);
    return CNF_OK;
    CNF_CATCH
}

int cnf_flow_backward_ex(cnf_plan* plan, const float* params, const float* xy, const float* zy, void* train_workspace,
                         int B, const float* global_count, float* dparams, cnf_layer_done_fn layer_done, void* user,
                         void* stream) {
    OptScope os_(plan ? &plan->p->opts : nullptr);
    if (!plan || !params || !xy || !zy || !train_workspace || !dparams || !global_count || B <= 0)
        return fail(CNF_E_INVALID, "null argument or B <= 0");
    CNF_TRY
    Plan& p = *plan->p;
    ensure_tables(p);
    flow_backward(p, params, xy, zy, train_workspace, B, 0.f, dparams, (hipStream_t)stream, global_count, layer_done,
                  user);
    return CNF_OK;
    CNF_CATCH
}

int cnf_coupling_backward(cnf_plan* plan, int layer, const float* params, const float* u, const float* dv, float* du,
                          float dlogdet, void* train_workspace, int B, float* dparams, void* stream) {
    OptScope os_(plan ? &plan->p->opts : nullptr);
    if (!plan || !params || !u || !dv || !du || !train_workspace || !dparams || B <= 0)
        return fail(CNF_E_INVALID, "null argument or B <= 0");
    CNF_TRY
    Plan& p = *plan->p;
    if (layer < 0 || layer >= (int)p.layers.size() || p.layers[layer].kind != CNF_LAYER_COUPLING)
        return fail(CNF_E_INVALID, "layer is not a coupling layer");
    if (du == dv || du == u) return fail(CNF_E_INVALID, "du must not alias u or dv");
    ensure_tables(p);
    coupling_layer_backward(p, p.layers[layer].ci, params, u, dv, du, dlogdet, train_workspace, B, dparams,
                            (hipStream_t)stream);
    return CNF_OK;
    CNF_CATCH
}

int cnf_adam_step(float* params, const float* grads, float* m, float* v, int64_t n, float lr, float beta_1,
                  float beta_2, float epsilon, int step, void* stream) {
    if (!params || !grads || !m || !v || n < 0 || step < 1) return fail(CNF_E_INVALID, "bad argument");
    CNF_TRY
    const double b1t = std::pow((double)beta_1, step), b2t = std::pow((double)beta_2, step);
    const float alpha = (float)((double)lr * std::sqrt(1.0 - b2t) / (1.0 - b1t));
    if (n > 0) launch_adam(params, grads, m, v, (long long)n, alpha, beta_1, beta_2, epsilon, (hipStream_t)stream);
    check_launch();
    return CNF_OK;
    CNF_CATCH
}

static void flow_inverse(Plan& p, const float* params, const float* aux, const float* zy, float* xy, void* workspace,
                         int B, hipStream_t stream);

int cnf_flow_inverse(cnf_plan* plan, const float* params, const float* aux, const float* zy, float* xy,
                     void* workspace, int B, void* stream) {
    OptScope os_(plan ? &plan->p->opts : nullptr);
    if (!plan || !params || !aux || !xy || !zy || !workspace || B <= 0)
        return fail(CNF_E_INVALID, "null argument or B <= 0");
    if (xy == zy) return fail(CNF_E_INVALID, "zy and xy must not alias (out-of-place only)");
    CNF_TRY
    flow_inverse(*plan->p, params, aux, zy, xy, workspace, B, (hipStream_t)stream);
    return CNF_OK;
    CNF_CATCH
}

}  // extern "C"

// cFlow.call(zy, -1) (:1774-1798) as a launch schedule
static void flow_inverse(Plan& p, const float* params, const float* aux, const float* zy, float* xy, void* workspace,
                         int B, hipStream_t stream) {
    if (!p.dry) ensure_tables(p);
    p.recorded.clear();
    Exec E{p, params, aux, (char*)workspace, p.layout(B), B, stream};
    const WsLayout& L = E.L;
    float* buf[2] = {E.at<float>(L.uv[0]), E.at<float>(L.uv[1])};
    const int nuv = (int)L.n_uv;
    const int* T = p.dtab(0);
    // squeeze/factor forward on zy (:1784-1788) == gather of the last block layout from xy positions
    int which = 0;
    {
        float* dst = buf[which];
        const int off = p.dev_final_orig, n = p.last_n;
        E.record("k_map_gather", 0, 8.0 * B * n,
                 [=](void* st) { launch_map_gather(zy, dst, T + off, n, nuv, n, B, (hipStream_t)st); });
    }
    const float* cur = buf[which];
    which ^= 1;
    // the first layer that launches anything (squeezes are folded into the boundary maps): the layer
    // the inverse ends with writes xy itself
    int first = 0;
    while (first < (int)p.layers.size() && p.layers[first].kind == CNF_LAYER_SQUEEZE) first++;
    // deferred inverse law (as the forward's, CoupPend::dir = -1): an LDS layer whose successor in
    // the inverse order (the previous layer by index) launches k_net_lds or the boundary maps leaves
    // its law to that kernel — no k_coupling launch for it
    const bool fuse = p.opts.fuse_coupling != 0;   // (debug option FUSE_COUPLING=0: a k_coupling per layer)
    CoupPend pend;
    bool have_pend = false;
    int bi = (int)p.boundaries.size() - 1;
    for (int li = (int)p.layers.size() - 1; li >= 0; li--) {
        const Layer& ly = p.layers[li];
        if (ly.kind == CNF_LAYER_COUPLING) {
            const Coupling& c = p.couplings[ly.ci];
            int nx = li - 1;
            while (nx >= 0 && p.layers[nx].kind == CNF_LAYER_SQUEEZE) nx--;
            const bool next_lds = nx >= 0 && p.layers[nx].kind == CNF_LAYER_COUPLING &&
                                  p.couplings[p.layers[nx].ci].use_lds;
            const bool next_maps = nx >= 0 && p.layers[nx].kind == CNF_LAYER_FACTOR;
            const bool defer = fuse && c.use_lds && (next_lds || next_maps);
            float* nxt = li == first ? xy : buf[which];
            CoupPend next;
            run_coupling(E, c, cur, nxt, nullptr, -1, have_pend ? &pend : nullptr, defer, &next);
            pend = next;
            have_pend = defer;
            cur = nxt;
            which ^= 1;
        } else if (ly.kind == CNF_LAYER_FACTOR) {
            // factor.backward (:294-329) + squeeze.backward (:191-217): rebuild the previous block
            // layout from the kept part (cur) and the factored part (read from zy at xy positions), one
            // k_map2 launch. With a pending coupling the kept part is read through it from u_k (the
            // other buffer), and v_k's own buffer (cur, never written) takes the result.
            const Boundary& b = p.boundaries[bi--];
            const bool last = li == first;
            float* prev = last ? xy : have_pend ? const_cast<float*>(cur) : buf[which];
            const bool flip = !have_pend;
            const int ncur = b.n_cur, nnext = b.n_next, nfac = b.n_fac;
            MapOp mk, mf;
            mk.src = cur, mk.dst = prev, mk.didx = T + b.dev_keep_src, mk.n = nnext, mk.ss = nnext, mk.ds = ncur;
            mf.src = zy, mf.dst = prev, mf.sidx = T + b.dev_fac_orig, mf.didx = T + b.dev_fac_src, mf.n = nfac;
            mf.ss = nuv, mf.ds = ncur;
            const CoupPend q = have_pend ? pend : CoupPend{};
            mk.pend = q.on;
            if (!p.dry && q.on && prev == q.u) throw std::logic_error("k_map2 would overwrite the u_k it reads");
            have_pend = false;
            E.record("k_map2", 0, 8.0 * B * (nnext + nfac),
                     [=](void* st) { launch_map2(mk, mf, LdReduce{}, q, B, (hipStream_t)st); });
            cur = prev;
            if (flip) which ^= 1;
        }
    }
    if (have_pend) throw std::logic_error("inverse: a deferred coupling was left pending");
    if (cur != xy) {   // (a schedule ending in a layout layer the maps did not cover)
        const float* src = cur;
        const size_t bytes = (size_t)B * nuv * 4;
        E.record("copy", 0, 2.0 * bytes, [=](void* st) {
            (void)hipMemcpyAsync(xy, src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)st);
        });
    }
    if (!p.dry) check_launch();
}

extern "C" {

int cnf_coupling_forward(cnf_plan* plan, int layer, const float* params, const float* aux, const float* u, float* v,
                         float* logdet_accum, void* workspace, int B, void* stream) {
    OptScope os_(plan ? &plan->p->opts : nullptr);
    if (!plan || !params || !aux || !u || !v || !workspace || B <= 0) return fail(CNF_E_INVALID, "null argument");
    CNF_TRY
    Plan& p = *plan->p;
    if (layer < 0 || layer >= (int)p.layers.size() || p.layers[layer].kind != CNF_LAYER_COUPLING)
        return fail(CNF_E_INVALID, "layer is not a coupling layer");
    if (u == v) return fail(CNF_E_INVALID, "u and v must not alias");
    ensure_tables(p);
    p.recorded.clear();
    Exec E{p, params, aux, (char*)workspace, p.layout(B), B, (hipStream_t)stream};
    double* ld = E.at<double>(E.L.ld);
    const Coupling& c = p.couplings[p.layers[layer].ci];
    run_coupling(E, c, u, v, logdet_accum ? ld : nullptr, +1);
    if (logdet_accum) {
        const int np = E.L.ld_parts;
        E.record("k_ld_reduce", 0, 0, [=](void* st) { launch_ld_reduce(ld, logdet_accum, B, 1, np, 1, (hipStream_t)st); });
    }
    check_launch();
    return CNF_OK;
    CNF_CATCH
}

int cnf_coupling_inverse(cnf_plan* plan, int layer, const float* params, const float* aux, const float* v, float* u,
                         void* workspace, int B, void* stream) {
    OptScope os_(plan ? &plan->p->opts : nullptr);
    if (!plan || !params || !aux || !u || !v || !workspace || B <= 0) return fail(CNF_E_INVALID, "null argument");
    CNF_TRY
    Plan& p = *plan->p;
    if (layer < 0 || layer >= (int)p.layers.size() || p.layers[layer].kind != CNF_LAYER_COUPLING)
        return fail(CNF_E_INVALID, "layer is not a coupling layer");
    if (u == v) return fail(CNF_E_INVALID, "u and v must not alias");
    ensure_tables(p);
    p.recorded.clear();
    Exec E{p, params, aux, (char*)workspace, p.layout(B), B, (hipStream_t)stream};
    run_coupling(E, p.couplings[p.layers[layer].ci], v, u, nullptr, -1);
    check_launch();
    return CNF_OK;
    CNF_CATCH
}

int cnf_squeeze(const float* in, float* out, int B, int H, int W, int C, int dir, void* stream) {
    if (!in || !out || B <= 0 || H <= 0 || W <= 0 || C <= 0) return fail(CNF_E_INVALID, "bad argument");
    if (dir > 0 && ((H % 2) || (W % 2))) return fail(CNF_E_INVALID, "u must have spatial dimensions divisible by 2.");
    if (dir < 0 && (C % 4)) return fail(CNF_E_INVALID, "v must have channel dimensions divisible by 4.");
    CNF_TRY
    launch_squeeze(in, out, B, H, W, C, dir > 0 ? 1 : -1, (hipStream_t)stream);
    check_launch();
    return CNF_OK;
    CNF_CATCH
}

int cnf_channel_copy(const float* in, int in_cs, int in_off, float* out, int out_cs, int out_off, int C, int B, int HW,
                     void* stream) {
    if (!in || !out || C < 0 || B <= 0 || HW <= 0 || in_off + C > in_cs || out_off + C > out_cs)
        return fail(CNF_E_INVALID, "bad channel window");
    if (C == 0) return CNF_OK;
    CNF_TRY
    launch_chcopy(in, in_cs, in_off, out, out_cs, out_off, C, (long long)B * HW, (hipStream_t)stream);
    check_launch();
    return CNF_OK;
    CNF_CATCH
}

int cnf_nll(const cnf_plan* plan, const float* xy, const float* zy, const float* logdet_per_image, float* per_image,
            float* sums, int B, void* stream) {
    OptScope os_(plan ? &plan->p->opts : nullptr);
    if (!plan || !xy || !zy || !logdet_per_image || !per_image || !sums || B <= 0)
        return fail(CNF_E_INVALID, "null argument");
    CNF_TRY
    Plan& p = *plan->p;
    ensure_tables(p);
    const cnf_flow_desc& d = p.desc;
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    hip_check(hipStreamIsCapturing((hipStream_t)stream, &cap), "hipStreamIsCapturing");
    const bool capturing = cap != hipStreamCaptureStatusNone;
    std::lock_guard<std::mutex> lk(*p.nll_mu);
    int slot = -1;
    for (size_t i = 0; i < p.nll_streams.size(); i++)
        if (p.nll_streams[i] == stream) slot = (int)i;
    if (slot < 0 && (int)p.nll_streams.size() < Plan::NLL_SLOTS) {
        p.nll_streams.push_back(stream);
        p.nll_ev.push_back(nullptr);
        p.nll_last.push_back(0);
        slot = (int)p.nll_streams.size() - 1;
    }
    if (slot < 0) {
        // every slot has its stream: take the least recently used one. Its counter is back at 0 once that
        // stream's last cnf_nll has completed, so this launch waits for it (stream-ordered, no host wait)
        slot = 0;
        for (int i = 1; i < Plan::NLL_SLOTS; i++)
            if (p.nll_last[i] < p.nll_last[slot]) slot = i;
        if (p.nll_ev[slot] != nullptr && hipEventQuery(p.nll_ev[slot]) != hipSuccess)
            hip_check(hipStreamWaitEvent((hipStream_t)stream, p.nll_ev[slot], 0), "hipStreamWaitEvent");
        else if (p.nll_ev[slot] == nullptr && capturing)
            throw std::runtime_error("cnf_nll: a 65th stream on one plan during graph capture (reuse needs an "
                                     "uncaptured call on the slot's stream first)");
        p.nll_streams[slot] = stream;
    }
    p.nll_last[slot] = ++p.nll_clock;
    unsigned* done = reinterpret_cast<unsigned*>(p.dev_table + p.host_table.size()) + slot;
    launch_nll(xy, zy, logdet_per_image, per_image, sums, done, B, d.io_h * d.io_w, d.io_d, d.x_d, d.lambda_y,
               (hipStream_t)stream);
    check_launch();
    if (!capturing) {   // (the slot's completion point, for a later reuse by another stream)
        if (p.nll_ev[slot] == nullptr)
            hip_check(hipEventCreateWithFlags(&p.nll_ev[slot], hipEventDisableTiming), "hipEventCreate");
        hip_check(hipEventRecord(p.nll_ev[slot], (hipStream_t)stream), "hipEventRecord");
    }
    return CNF_OK;
    CNF_CATCH
}

// diagnostic: phase stamps of the last CNF_STAMPS=1 k_net_lds launch (s_memrealtime, 100 MHz)
// ---- TOYcINN -------------------------------------------------------------------------------
static int64_t toy_net_floats(int n1, int n2, int H, int L) {
    return (int64_t)n1 * H + H + (int64_t)L * (H * H + H) + (int64_t)H * n2 + n2;
}

static void toy_check(const cnf_toy_desc* d) {
    if (!d) throw std::invalid_argument("null toy descriptor");
    if (d->io_shape != 3) throw std::invalid_argument("TOYcINN masks are defined for io_shape == 3 only");
    if (d->x_d < 1 || d->x_d > 2) throw std::invalid_argument("x_d must be 1 or 2");
    if (d->num_coupling_layers < 1 || d->num_coupling_layers > TOY_MAXL)
        throw std::invalid_argument("num_coupling_layers must be in [1, 128]");
    if (d->intermediate_dims < 1 || d->intermediate_dims > 64) throw std::invalid_argument("intermediate_dims must be in [1, 64]");
    if (d->num_layers < 0) throw std::invalid_argument("num_layers must be >= 0");
    if (!d->mask_indices) throw std::invalid_argument("mask_indices is required");
    std::vector<int> seen(d->num_coupling_layers, 0);
    for (int i = 0; i < d->num_coupling_layers; i++) {
        const int j = d->mask_indices[i];
        if (j < 0 || j >= d->num_coupling_layers || seen[j]++) throw std::invalid_argument("mask_indices must be a permutation");
    }
}

int64_t cnf_toy_num_params(const cnf_toy_desc* d) {
    CNF_TRY
    toy_check(d);
    int64_t n = 0;
    for (int j = 0; j < d->num_coupling_layers; j++) {
        const int n1 = (j % 6) < 3 ? 1 : 2;
        n += 2 * toy_net_floats(n1, 3 - n1, d->intermediate_dims, d->num_layers);
    }
    return n;
    CNF_CATCH
}

int cnf_toy_call(const cnf_toy_desc* d, const float* params, const float* u, float* v, float* log_detJ,
                 float* per_sample, int B, int direction, void* stream) {
    CNF_TRY
    toy_check(d);
    if (!params || !u || !v || B < 0) return fail(CNF_E_INVALID, "null pointer or negative batch");
    if (direction != 1 && direction != -1) return fail(CNF_E_INVALID, "direction must be +1 or -1");
    if (u == v) return fail(CNF_E_INVALID, "u and v must not alias");
    if (B == 0) return CNF_OK;
    ToyArgs a;
    std::memset(&a, 0, sizeof(a));
    a.params = params;
    a.u = u;
    a.v = v;
    a.log_detJ = direction < 0 ? log_detJ : nullptr;
    a.per_sample = direction < 0 ? per_sample : nullptr;
    a.B = B;
    a.nl = d->num_coupling_layers;
    a.H = d->intermediate_dims;
    a.L = d->num_layers;
    a.x_d = d->x_d;
    a.dir = direction;
    a.lambda_y = d->lambda_y;
    int64_t off = 0, maxn = 0;
    for (int j = 0; j < a.nl; j++) {
        a.order[j] = d->mask_indices[j];
        a.net_off[j] = (int)off;
        const int n1 = (j % 6) < 3 ? 1 : 2;
        const int64_t n = 2 * toy_net_floats(n1, 3 - n1, a.H, a.L);
        off += n;
        maxn = std::max(maxn, n);
    }
    a.net_off[a.nl] = (int)off;
    if (maxn * 4 > 160 * 1024) return fail(CNF_E_INVALID, "toy coupling networks exceed the 160 KiB LDS staging budget");
    launch_toy(a, (int)maxn, (hipStream_t)stream);
    hip_check(hipGetLastError(), "k_toy");
    return CNF_OK;
    CNF_CATCH
}

int cnf_toy_nll_sums(const float* per_sample, float* sums, int B, void* stream) {
    CNF_TRY
    if (!per_sample || !sums || B < 1) return fail(CNF_E_INVALID, "null pointer or empty batch");
    launch_nll_sums(per_sample, sums, B, (hipStream_t)stream);
    hip_check(hipGetLastError(), "k_nll_sums");
    return CNF_OK;
    CNF_CATCH
}

// shape words of coupling `coupling`'s k_net_lds launch (0 if the layer is streamed); host only, used
// by csrc/gen_netlds_shapes.py to generate the shape-specialised instantiations' table
int cnf_debug_netlds_shape(const cnf_plan* plan, int coupling, int* words, int cap) {
    OptScope os_(plan ? &plan->p->opts : nullptr);
    if (!plan || !words || cap < NETSHAPE_WORDS) return -1;
    const Plan& p = *plan->p;
    if (coupling < 0 || coupling >= (int)p.couplings.size()) return -1;
    const Coupling& c = p.couplings[coupling];
    if (!c.use_lds) return 0;
    NetLdsArgs a;
    if (netlds_setup(p, c, a) == 0) return 0;
    netshape_words(a, words);
    return NETSHAPE_WORDS;
}
int cnf_debug_netlds_nshapes() { return netlds_num_shapes(); }

// k_pw launch shapes of a B-image forward, from a host-only dry run (nothing is launched or
// dereferenced: the tensors are placeholder addresses); returns the number of words written
int cnf_debug_pw_shapes(cnf_plan* plan, int B, int* words, int cap);
// k_gc launch shapes of a B-image forward (host-only dry run, as cnf_debug_pw_shapes)
int cnf_debug_gc_launch_shapes(cnf_plan* plan, int B, int* words, int cap) {
    OptScope os_(plan ? &plan->p->opts : nullptr);
    if (!plan || !words || B <= 0) return -1;
    const int n = cnf_debug_pw_shapes(plan, B, words, cap);   // the dry run also records the k_gc shapes
    if (n < 0) return -1;
    const std::vector<GcShape>& g = plan->p->gc_launch;
    if ((int64_t)g.size() * GCSHAPE_WORDS > cap) return -1;
    for (size_t i = 0; i < g.size(); i++) std::memcpy(words + i * GCSHAPE_WORDS, &g[i], sizeof(GcShape));
    return (int)g.size() * GCSHAPE_WORDS;
}

// launch names of a B-image forward (direction +1) or inverse (-1) from a host-only dry run, one per
// line into out (cap bytes, NUL-terminated); returns the number of launches, -1 on error
int cnf_debug_schedule(cnf_plan* plan, int B, int direction, char* out, int cap) {
    OptScope os_(plan ? &plan->p->opts : nullptr);
    if (!plan || !out || cap <= 0 || B <= 0 || (direction != 1 && direction != -1)) return -1;
    Plan& p = *plan->p;
    CNF_TRY
    p.dry = true;
    p.dry_launches.clear();
    char* fake = reinterpret_cast<char*>(uintptr_t(1) << 40);   // never dereferenced
    const float* f = reinterpret_cast<const float*>(fake);
    float* g = reinterpret_cast<float*>(fake + (1 << 20));        // a distinct output address
    try {
        if (direction > 0)
            flow_forward(p, f, f, f, g, g, fake, B, nullptr, false);
        else
            flow_inverse(p, f, f, f, g, fake, B, nullptr);
    } catch (...) {
        p.dry = false;
        throw;
    }
    p.dry = false;
    p.recorded.clear();
    std::string s;
    for (const std::string& n : p.dry_launches) s += n + "\n";
    if ((int)s.size() + 1 > cap) return -1;
    std::memcpy(out, s.c_str(), s.size() + 1);
    return (int)p.dry_launches.size();
    CNF_CATCH
}

int cnf_debug_pw_shapes(cnf_plan* plan, int B, int* words, int cap) {
    OptScope os_(plan ? &plan->p->opts : nullptr);
    if (!plan || !words || B <= 0) return -1;
    Plan& p = *plan->p;
    CNF_TRY
    p.dry = true;
    p.pw_shapes.clear();
    p.gc_launch.clear();
    char* fake = reinterpret_cast<char*>(uintptr_t(1) << 40);   // never dereferenced
    try {
        flow_forward(p, (const float*)fake, (const float*)fake, (const float*)fake, (float*)fake, (float*)fake, fake, B,
                     nullptr, false);
    } catch (...) {
        p.dry = false;
        throw;
    }
    p.dry = false;
    p.recorded.clear();
    const int n = (int)p.pw_shapes.size() * PWSHAPE_WORDS;
    if (n > cap) return -1;
    for (size_t i = 0; i < p.pw_shapes.size(); i++)
        std::memcpy(words + i * PWSHAPE_WORDS, &p.pw_shapes[i], sizeof(PwShape));
    return n;
    CNF_CATCH
}

int cnf_debug_pw_nshapes() { return pw_num_shapes(); }
int cnf_debug_pw_words() { return PWSHAPE_WORDS; }

// shape words of coupling `coupling`'s k_gc launches, one GcShape per group (0 if it has none)
int cnf_debug_gc_shape(const cnf_plan* plan, int coupling, int* words, int cap) {
    OptScope os_(plan ? &plan->p->opts : nullptr);
    if (!plan || !words) return -1;
    const Plan& p = *plan->p;
    if (coupling < 0 || coupling >= (int)p.couplings.size()) return -1;
    const Coupling& c = p.couplings[coupling];
    if (c.use_lds || !c.gc_fused) return 0;
    if (cap < GCSHAPE_WORDS * (int)c.gcg.size()) return -1;
    int n = 0;
    for (const Coupling::GcGroup& gg : c.gcg) {
        GcShape s;
        std::memset(&s, 0, sizeof(s));
        for (size_t k = 0; k < gg.br.size(); k++) s.br[k] = gg.gcb[k];
        s.nbr = (int)gg.br.size();
        s.H = c.hc;
        s.W = c.wc;
        s.in_cs = c.t1_cs;   // as run_coupling launches it
        s.out_cs = c.t2_cs;
        s.TH = gg.TH;
        s.TW = gg.TW;
        s.tiles_x = gg.tiles_x;
        s.tiles_per_img = gg.tiles();
        s.ps = gg.ps;
        s.nbk = gg.nbk;
        s.tpp = gg.tpp;
        s.nw = gg.nw;
        s.pd = gg.pd;
        s.band_bytes = gg.band_bytes;
        s.lnst = p.desc.layer_norm ? 3 : 0;   // the forward's k_gc: LN2 on load and LN3 partials iff LayerNorm
        std::memcpy(words + n, &s, sizeof(s));
        n += GCSHAPE_WORDS;
    }
    return n;
}
int cnf_debug_gc_words() { return GCSHAPE_WORDS; }

// t1 layout of a coupling (Coupling::t1_map): [compact, floats per pixel of the image, then per branch
// (window offset of pixel 0, pixel stride, cin_off, cin), then 128 words of t1_map (compact only)]
// t2 layout of a coupling (Coupling::t2_*): [mapped, floats per pixel of the image, gc, then per branch
// (slice offset of pixel 0, pixel stride, out_off, cout), then conv_b's quad map (gc / 4 pairs, mapped only)]
int cnf_debug_t2_layout(const cnf_plan* plan, int coupling, int* words, int cap) {
    OptScope os_(plan ? &plan->p->opts : nullptr);
    if (!plan || !words) return -1;
    const Plan& p = *plan->p;
    if (coupling < 0 || coupling >= (int)p.couplings.size()) return -1;
    const Coupling& c = p.couplings[coupling];
    std::vector<int> w = {c.t2_mapped ? 1 : 0, c.t2_cs, c.gc};
    for (size_t bi = 0; bi < c.br.size(); bi++) {
        w.push_back(bi < c.t2_off.size() ? c.t2_off[bi] : -1);
        w.push_back(bi < c.t2_pcs.size() ? c.t2_pcs[bi] : -1);
        w.push_back(c.br[bi].out_off);
        w.push_back(c.br[bi].cout);
    }
    w.insert(w.end(), c.t2_qmap.begin(), c.t2_qmap.end());
    if ((int)w.size() > cap) return -1;
    std::memcpy(words, w.data(), w.size() * sizeof(int));
    return (int)w.size();
}

int cnf_debug_t1_layout(const cnf_plan* plan, int coupling, int* words, int cap) {
    OptScope os_(plan ? &plan->p->opts : nullptr);
    if (!plan || !words) return -1;
    const Plan& p = *plan->p;
    if (coupling < 0 || coupling >= (int)p.couplings.size()) return -1;
    const Coupling& c = p.couplings[coupling];
    std::vector<int> w = {c.t1_compact ? 1 : 0, c.t1_cs};
    for (size_t bi = 0; bi < c.br.size(); bi++) {
        w.push_back(bi < c.t1_off.size() ? c.t1_off[bi] : -1);
        w.push_back(bi < c.t1_pcs.size() ? c.t1_pcs[bi] : -1);
        w.push_back(c.br[bi].cin_off);
        w.push_back(c.br[bi].cin);
    }
    w.insert(w.end(), c.t1_map.begin(), c.t1_map.end());
    if ((int)w.size() > cap) return -1;
    std::memcpy(words, w.data(), w.size() * sizeof(int));
    return (int)w.size();
}

int cnf_debug_read_stamps(long long* out, int n) { return read_stamps(out, n); }
int cnf_debug_read_bwd_stamps(long long* out, int n) { return read_bwd_stamps(out, n); }
int cnf_debug_read_cycles(long long* out, int n) { return read_cycles(out, n); }
int cnf_debug_read_gc_stamps(long long* out, int n) { return read_gc_stamps(out, n); }
int cnf_debug_read_pw_stamps(long long* out) { return read_pw_stamps(out); }

int cnf_plan_num_recorded_launches(const cnf_plan* plan) { return plan ? (int)plan->p->recorded.size() : -1; }

int cnf_plan_recorded_launch_info(const cnf_plan* plan, int i, char* name, int name_cap, double* flops,
                                  double* bytes) {
    OptScope os_(plan ? &plan->p->opts : nullptr);
    if (!plan) return fail(CNF_E_INVALID, "null plan");
    const Plan& p = *plan->p;
    if (i < 0 || i >= (int)p.recorded.size()) return fail(CNF_E_INVALID, "launch index out of range");
    if (name && name_cap > 0) std::snprintf(name, (size_t)name_cap, "%s", p.recorded[i].name.c_str());
    if (flops) *flops = p.recorded[i].flops;
    if (bytes) *bytes = p.recorded[i].bytes;
    return CNF_OK;
}

int cnf_plan_set_launch_timing(cnf_plan* plan, int on) {
    OptScope os_(plan ? &plan->p->opts : nullptr);
    if (!plan) return fail(CNF_E_INVALID, "null plan");
    plan->p->timing = on != 0;
    return CNF_OK;
}

int cnf_plan_launch_time_ms(const cnf_plan* plan, int i, float* ms) {
    OptScope os_(plan ? &plan->p->opts : nullptr);
    if (!plan || !ms) return fail(CNF_E_INVALID, "null argument");
    const Plan& p = *plan->p;
    if (i < 0 || i >= (int)p.recorded.size()) return fail(CNF_E_INVALID, "launch index out of range");
    if (!p.recorded[i].timed) {   // not a kernel (a copy), or the call ran without launch timing
        *ms = 0.f;
        return CNF_OK;
    }
    CNF_TRY
    hip_check(hipEventSynchronize(p.ev[2 * i + 1]), "hipEventSynchronize");
    hip_check(hipEventElapsedTime(ms, p.ev[2 * i], p.ev[2 * i + 1]), "hipEventElapsedTime");
    return CNF_OK;
    CNF_CATCH
}

int64_t cnf_plan_weight_map(const cnf_plan* plan, int which, int64_t* out, int64_t cap) {
    OptScope os_(plan ? &plan->p->opts : nullptr);
    if (!plan || (which != 0 && which != 1)) return fail(CNF_E_INVALID, "null plan or which not in {0, 1}");
    const std::vector<int64_t>& m = which == 0 ? plan->p->aux_map : plan->p->bw_map;
    if (out)
        for (int64_t i = 0; i < std::min<int64_t>(cap, (int64_t)m.size()); i++) out[i] = m[i];
    return (int64_t)m.size();
}

int cnf_plan_relaunch(cnf_plan* plan, int i, void* stream) {
    OptScope os_(plan ? &plan->p->opts : nullptr);
    if (!plan) return fail(CNF_E_INVALID, "null plan");
    Plan& p = *plan->p;
    if (i < 0 || i >= (int)p.recorded.size()) return fail(CNF_E_INVALID, "launch index out of range");
    CNF_TRY
    p.recorded[i].relaunch(stream);
    check_launch();
    return CNF_OK;
    CNF_CATCH
}

}  // extern "C"
