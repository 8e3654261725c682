/*
 * The batched BF16 training plan (see bplan.h): configuration, buffers and the kernel
 * sequence of every step structure, in one place for the C engine and the Python binding.
 */
#include "bplan.h"

#include <libhpnn.h>
#include <libhpnn/comm.h>
#include <libhpnn/devmem.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

namespace hpnn {

namespace {

inline int pad_to(int v, int m) { return (v + m - 1) / m * m; }

bool env_off(const char *name) {
    const char *e = getenv(name);
    return e && e[0] == '0';
}

size_t dtype_bytes(int dt) { return dt == BD_F32 || dt == BD_I32 ? 4 : (dt == BD_BF16 ? 2 : 1); }

/* first-layer input widths of the fused MNIST-shape fronts (kernels_mlp3x.hip / _mlp3t.hip) */
bool in_list(int v, std::initializer_list<int> l) {
    for (int x : l)
        if (x == v) return true;
    return false;
}

constexpr int TILE_T = 256; /* samples per mlp3_tile tile */
constexpr int TILE_W = 128; /* samples per wide2_front tile */

}  // namespace

size_t BufSpec::bytes() const {
    size_t n = dtype_bytes(dtype);
    for (int i = 0; i < ndim; i++) n *= (size_t)shape[i];
    return n;
}

/* split-K factor of the weight-gradient GEMM (N x K over Bp batch rows).
 * 256 x 256 tiles: enough splits for the 8-phase TN kernel (>= 256 workgroups, an even number
 * of 64-row units per split; RRUFF's 4096 -> 256 layer over 16384 rows: 16 splits, 162-164
 * us per step vs 171-173 with 4 on the 128 x 128 kernel).  Otherwise about one workgroup per
 * CU (256 on MI355X) so every CU streams the same share (the kernels take uneven 64-row units
 * per split), >= HPNN_TN_ROWS (512) batch rows per split, a multiple of 8 for the XCD-aware
 * block order: MNIST's G0 (128 x 800 over 65536 rows) 48 splits, measured fastest among
 * 24-64 (profiles/r3/s7_g0_splits_ab.txt).  HPNN_TN_SPLITS forces a value (tuning). */
int BPlan::pick_splits(int Np, int Kp, int Bp) {
    static const int forced = [] {
        const char *e = getenv("HPNN_TN_SPLITS");
        return e ? atoi(e) : 0;
    }();
    if (forced > 0) {
        if (Bp % 64) return 1;
        const int m = Bp / 64;
        return forced < m ? forced : m;
    }
    static const bool tn8 = !env_off("HPNN_TN_8PH");
    if (tn8 && Np % 256 == 0 && Kp % 256 == 0 && Bp % 128 == 0) {
        const int t8 = (Np / 256) * (Kp / 256), units = Bp / 64, s0 = (256 + t8 - 1) / t8;
        for (int s8 = s0; s8 <= 2 * s0; s8++)
            if (units % s8 == 0 && (units / s8) % 2 == 0) return s8;
    }
    const int tn = Np % 128 == 0 ? 128 : (Np % 64 == 0 ? 64 : 32);
    const int tm = Kp % 128 == 0 ? 128 : (Kp % 160 == 0 ? 160 : (Kp % 96 == 0 ? 96 : (Kp % 64 == 0 ? 64 : 32)));
    const int tiles = (Np / tn) * (Kp / tm);
    static const int rows = [] {
        const char *e = getenv("HPNN_TN_ROWS");
        return e && atoi(e) > 0 ? atoi(e) : 512;
    }();
    int s = (256 + tiles / 2) / (tiles > 0 ? tiles : 1);
    const int maxs = Bp / rows;
    if (s > maxs) s = maxs;
    if (s >= 8) s -= s % 8;
    return s < 1 ? 1 : s;
}

int BPlan::configure(const int *sizes, int n_layers, int net_type, int batch_size, bool momentum_, int fused,
                     const int *splits, int mid_grid_req, bool device, std::string *err) {
    auto fail = [&](int code, const std::string &m) {
        if (err) *err = m;
        return code;
    };
    if (n_layers < 1 || n_layers > 15 || batch_size < 1) return fail(-1, "1..15 weight layers and batch >= 1");
    for (int l = 0; l <= n_layers; l++)
        if (sizes[l] < 1) return fail(-1, "layer sizes must be >= 1");
    L = n_layers;
    type = net_type;
    batch = batch_size;
    momentum = momentum_;
    on_device = device;
    n_out = sizes[L];
    for (int l = 0; l < L; l++) {
        M[l] = sizes[l];
        N[l] = sizes[l + 1];
        Kp[l] = pad_to(M[l], 32);
        Np[l] = pad_to(N[l], 32);
    }
    Bp = pad_to(batch, 128);
    /* eligibility of the fused step structures */
    const bool mnist = L == 3 && Np[0] == 128 && Np[1] == 64 && Np[2] == 32;
    const bool x_ok = mnist && in_list(Kp[0], {256, 512, 800, 832, 896});
    const bool t_shape = mnist && in_list(Kp[0], {256, 800});
    const bool w_ok = L == 2 && Np[0] == 256 && Np[1] == 256 && Kp[0] == 4096;
    char m = 0;
    if (fused < 0) {
        /* HPNN_TILE=0 / HPNN_WIDE=0: the next structure down (A/B measurements) */
        if (t_shape && Bp % TILE_T == 0 && !env_off("HPNN_TILE")) m = 't';
        else if (x_ok) m = 'x';
        else if (mnist) m = 'm';
        else if (w_ok && !env_off("HPNN_WIDE")) m = 'w';
    } else if (fused > 0) {
        const bool ok = fused == 't' ? t_shape : fused == 'x' ? x_ok : fused == 'm' ? mnist : fused == 'w' ? w_ok : false;
        if (!ok) return fail(-2, std::string("fused mode '") + (char)fused + "' not available for these dims");
        m = (char)fused;
    }
    mode = m;
    if (mode == 't') Bp = pad_to(Bp, TILE_T); /* whole tiles; padded rows are zero and masked by n_valid */
    for (int l = 0; l < L; l++) S[l] = (splits && splits[l] > 0) ? splits[l] : pick_splits(Np[l], Kp[l], Bp);
    /* modes t / x: the first-layer gradient runs on the fused G0 launch's own tiles (160 or 80
     * feature columns x 128): about one workgroup per CU of THOSE tiles */
    if ((mode == 't' || mode == 'x') && !(splits && splits[0] > 0) && !getenv("HPNN_TN_SPLITS")) {
        const int tiles = hpnn_g0_tiles(1, Np[0], Kp[0]);
        if (tiles > 0) {
            int s0 = (256 + tiles / 2) / tiles;
            if (s0 > Bp / 512) s0 = Bp / 512;
            if (s0 >= 8) s0 -= s0 % 8;
            S[0] = s0 < 1 ? 1 : s0;
        }
    }
    slab_f = hpnn_mlp3_slab_floats();
    if (mode == 't') mid_grid = device ? hpnn_mlp3_tile_grid(Bp, 0) : 1;
    else if (mode == 'x') mid_grid = device ? hpnn_mlp3_fused_grid(Bp, 0) : 1;
    else if (mode == 'm') mid_grid = device ? (Bp / 64 < mid_grid_req ? Bp / 64 : mid_grid_req) : 1;
    else mid_grid = 0;
    if (mode && mode != 'w' && mid_grid < 1) return fail(-3, "no grid for the fused front");
    mid_groups = mid_grid < 16 ? (mid_grid > 0 ? mid_grid : 1) : 16;
    wide_ksplit = (mode == 'w' && device) ? hpnn_wide2_ksplit(Bp, Kp[0]) : 1;
    if (mode == 'w' && wide_ksplit < 1) return fail(-3, "wide front: unsupported batch");
    goff[0] = 0;
    for (int l = 0; l < L; l++) goff[l + 1] = goff[l] + (size_t)Np[l] * Kp[l];

    /* buffer table */
    specs.clear();
    auto add = [&](const char *name, int layer, int dt, std::initializer_list<long> shape, bool zero) {
        BufSpec b;
        b.name = name;
        b.layer = layer;
        b.dtype = dt;
        b.ndim = (int)shape.size();
        int i = 0;
        for (long v : shape) b.shape[i++] = v;
        for (; i < 4; i++) b.shape[i] = 1;
        b.zero = zero;
        specs.push_back(b);
    };
    for (int l = 0; l < L; l++) {
        add("W32", l, BD_F32, {Np[l], Kp[l]}, true);
        if (momentum) add("V32", l, BD_F32, {Np[l], Kp[l]}, true);
        add("Wb", l, BD_BF16, {Np[l], Kp[l]}, true);
        add("Wt", l, BD_BF16, {Kp[l], Np[l]}, true);
        add("slab", l, BD_F32, {S[l], Np[l], Kp[l]}, false);
        if (l < L - 1) add("H", l, BD_BF16, {Bp, Np[l]}, false);
        add("D", l, BD_BF16, {Bp, Np[l]}, false);
    }
    add("gflat", -1, BD_F32, {(long)goff[L]}, true);
    add("Z", -1, BD_F32, {Bp, Np[L - 1]}, false);
    add("stats", -1, BD_F32, {HPNN_STAT_SLOTS, HPNN_STAT_STRIDE}, true);
    add("lab0", -1, BD_I32, {Bp}, true);
    if (mode == 't' || mode == 'x' || mode == 'm') {
        add("midslab", -1, BD_F32, {mid_grid, slab_f}, false);
        add("midtmp", -1, BD_F32, {16, slab_f}, false);
    }
    if (mode == 't' || mode == 'x') {
        add("W0f", -1, BD_BF16, {(long)Np[0] * Kp[0]}, true);
        add("g0cnt", -1, BD_I32, {HPNN_G0CNT_WORDS}, true); /* fused G0 step: tile counters + error word */
        /* its XCD-local first reduction level (HPNN_G0_XCD=1): protocol words + 8 group partials */
        add("g0xw", -1, BD_I32, {HPNN_G0X_WORDS}, true);
        add("g0xs", -1, BD_F32, {8, Np[0], Kp[0]}, false);
    }
    if (mode == 'w') {
        const long pb = wide_ksplit == 2 ? hpnn_wide2_pbuf_bytes(Bp) : 16;
        add("wpbuf", -1, BD_F32, {pb / 4}, false);
        add("wwords", -1, BD_I32, {2L * (Bp / TILE_W) + 4}, true);
        /* fused split-K TN steps: a ticket block of its own per layer (the counters are monotonic
         * and the S of each layer differs), then the error word */
        add("tncnt", -1, BD_I32, {(long)(L + 1) * 1024}, true);
    }
    return 0;
}

void *BPlan::buf(const char *name, int layer) const {
    for (size_t i = 0; i < specs.size() && i < ptr_.size(); i++)
        if (specs[i].layer == layer && specs[i].name == name) return ptr_[i];
    return nullptr;
}

void BPlan::name_pointers() {
    for (int l = 0; l < L; l++) {
        W32[l] = (float *)buf("W32", l);
        V32[l] = (float *)buf("V32", l);
        Wb[l] = buf("Wb", l);
        Wt[l] = buf("Wt", l);
        slab[l] = (float *)buf("slab", l);
        H[l] = buf("H", l);
        D[l] = buf("D", l);
    }
    gflat = (float *)buf("gflat");
    Z = (float *)buf("Z");
    stats = (float *)buf("stats");
    lab0 = (int *)buf("lab0");
    midslab = (float *)buf("midslab");
    midtmp = (float *)buf("midtmp");
    W0f = buf("W0f");
    g0cnt = (unsigned int *)buf("g0cnt");
    g0xw = (unsigned int *)buf("g0xw");
    g0xs = (float *)buf("g0xs");
    tncnt = (unsigned int *)buf("tncnt");
    wpbuf = (float *)buf("wpbuf");
    wwords = (unsigned int *)buf("wwords");
}

int BPlan::allocate(hipStream_t s) {
    ptr_.assign(specs.size(), nullptr);
    owns_ = true;
    for (size_t i = 0; i < specs.size(); i++) {
        if (hpnn_dev_malloc(&ptr_[i], specs[i].bytes()) != hipSuccess) return -7;
        if (specs[i].zero && hipMemsetAsync(ptr_[i], 0, specs[i].bytes(), s) != hipSuccess) return -7;
    }
    name_pointers();
    return 0;
}

int BPlan::bind(void *const *ptrs) {
    ptr_.assign(ptrs, ptrs + specs.size());
    owns_ = false;
    name_pointers();
    return 0;
}

BPlan::~BPlan() {
    if (digest_) hpnn_dev_free(digest_);
    if (!owns_) return;
    for (void *p : ptr_)
        if (p) hpnn_dev_free(p);
}

/* ------------------------------------------------------------------ launches */
int BPlan::cast_weights(hipStream_t s) {
    for (int l = 0; l < L; l++) {
        int r;
        if (l == 0 && W0f) { /* an lr = 0 update is exactly a cast, and writes the fragment-major copy */
            hpnn_upd_layer c0 = {W32[0], nullptr, W32[0], 0, Wb[0], Wt[0], W0f, 1, Np[0], Kp[0]};
            r = hpnn_sgd_update_multi(&c0, 1, 0.f, 0.f, 0.f, 0, s);
        } else {
            r = hpnn_cast_weights(W32[l], Wb[l], Wt[l], Np[l], Kp[l], s);
        }
        if (r) return r;
    }
    return 0;
}

int BPlan::zero_stats(hipStream_t s) {
    return hipMemsetAsync(stats, 0, (size_t)HPNN_STAT_SLOTS * HPNN_STAT_STRIDE * 4, s) == hipSuccess ? 0 : -7;
}

int BPlan::forward(const void *X, hipStream_t s) {
    for (int l = 0; l < L; l++) {
        const void *A = l ? H[l - 1] : X;
        const bool last = l == L - 1;
        int r = hpnn_gemm_nt_bf16(A, Kp[l], Wb[l], Kp[l], last ? (void *)Z : H[l], Np[l], nullptr, 0, Bp, Np[l], Kp[l],
                                  last ? HPNN_EPI_NONE : HPNN_EPI_ACT, last ? 1 : 0, s);
        if (r) return r;
    }
    return 0;
}

int BPlan::output(const int *labels, const float *T, int ldt, int n_valid, float *O, int ldo, bool with_stats,
                  hipStream_t s) {
    return hpnn_output_delta(Z, Np[L - 1], T, ldt, labels, 1.f, type == 2 ? 0.f : -1.f, D[L - 1], Np[L - 1], O, ldo,
                             with_stats ? stats : nullptr, with_stats ? (unsigned int *)(stats + 1) : nullptr, Bp,
                             n_valid, n_out, type, s);
}

/* D[l-1] = (D[l] . W_l) * f'(H[l-1]) with the pre-update W_l^T ([Kp[l] x Np[l]]) */
int BPlan::backward_layer(int l, hipStream_t s) {
    if (l < 1 || l >= L) return -1;
    if (nn_bwd[l])
        return hpnn_gemm_nn_bf16(D[l], Np[l], Wb[l], Kp[l], D[l - 1], Np[l - 1], H[l - 1], Np[l - 1], Bp, Np[l - 1],
                                 Np[l], HPNN_EPI_DACT, 0, s);
    return hpnn_gemm_nt_bf16(D[l], Np[l], Wt[l], Np[l], D[l - 1], Np[l - 1], H[l - 1], Np[l - 1], Bp, Np[l - 1], Np[l],
                             HPNN_EPI_DACT, 0, s);
}

const void *BPlan::fm_input(const XIn &x) const {
    if (mode == 't') return x.x;
    if (mode == 'x') return x.xg;
    return nullptr;
}

int BPlan::grad_layer(int l, const XIn &x, bool reduce, hipStream_t s) {
    const long nw = (long)Np[l] * Kp[l];
    const void *fm = l == 0 ? fm_input(x) : nullptr;
    int r;
    if (fm) { /* delta1 came fragment-major from the fused front */
        r = hpnn_gemm_fm_direct(D[0], fm, x.u8, x.u8 ? x.scale : 1.f, slab[0], Kp[0], Np[0], Kp[0], Bp, S[0], s);
    } else {
        if (l == 0 && mode == 't') return -2; /* the tile path's input is fragment-major only */
        const void *Hin = l ? H[l - 1] : x.x;
        g16_used[l] = false;
        if (reduce && S[l] == 1 && g16[l] &&
            hpnn_gemm_tn8_bf16out(D[l], Np[l], Hin, Kp[l], g16[l], Kp[l], Np[l], Kp[l], Bp, s) == 0) {
            g16_used[l] = true; /* BF16 straight into the exchange's send buffer */
            return 0;
        }
        if (reduce && S[l] == 1) /* one split: the GEMM writes the all-reduce bucket itself */
            return hpnn_gemm_tn_bf16(D[l], Np[l], Hin, Kp[l], gflat + goff[l], Kp[l], Np[l], Kp[l], Bp, 1, s);
        r = hpnn_gemm_tn_bf16(D[l], Np[l], Hin, Kp[l], slab[l], Kp[l], Np[l], Kp[l], Bp, S[l], s);
    }
    if (!r && reduce) r = hpnn_reduce_slabs(slab[l], S[l], nw, nw, gflat + goff[l], s);
    return r;
}

int BPlan::update_layer(int l, float lr, float alpha, float scale, bool from_g, hipStream_t s) {
    const float *G = from_g ? gflat + goff[l] : slab[l];
    const int Sn = from_g ? 1 : S[l];
    const long gs = from_g ? 0 : (long)Np[l] * Kp[l];
    if (l == 0 && W0f) {
        hpnn_upd_layer u = {W32[0], V32[0], G, gs, Wb[0], Wt[0], W0f, Sn, Np[0], Kp[0]};
        return hpnn_sgd_update_multi(&u, 1, lr, alpha, scale, momentum ? 1 : 0, s);
    }
    return hpnn_sgd_update(W32[l], V32[l], G, Sn, gs, Wb[l], Wt[l], Np[l], Kp[l], lr, alpha, scale, momentum ? 1 : 0,
                           s);
}

int BPlan::front(const XIn &x, const int *labels, const float *T, int ldt, int n_valid, hipStream_t s) {
    const float t_lo = type == 2 ? 0.f : -1.f;
    unsigned int *hits = (unsigned int *)(stats + 1);
    int r;
    switch (mode) {
    case 't':
        r = hpnn_mlp3_tile(x.x, x.u8, x.u8 ? x.scale : 1.f, Kp[0], W0f, Wb[1], Wb[2], Wt[2], labels, T, ldt, 1.f, t_lo,
                           D[0], midslab, stats, hits, Bp, n_valid, n_out, type, mid_grid, s);
        return r > 0 ? 0 : (r ? r : -1);
    case 'x':
        r = hpnn_mlp3_fused(x.x, Kp[0], Kp[0], W0f, Wb[1], Wb[2], labels, T, ldt, 1.f, t_lo, D[0], midslab, stats, hits,
                            Bp, n_valid, n_out, type, mid_grid, fm_input(x) ? 1 : 0, s);
        return r > 0 ? 0 : (r ? r : -1);
    case 'm':
        r = hpnn_gemm_nt_bf16(x.x, Kp[0], Wb[0], Kp[0], H[0], Np[0], nullptr, 0, Bp, Np[0], Kp[0], HPNN_EPI_ACT, 0, s);
        if (r) return r;
        return hpnn_mlp3_mid(H[0], Wb[1], Wt[1], Wb[2], Wt[2], labels, T, ldt, 1.f, t_lo, D[0], midslab, stats, hits,
                             Bp, n_valid, n_out, type, Np[0], Np[1], Np[2], mid_grid, s);
    case 'w': {
        hpnn_wide2_args a;
        memset(&a, 0, sizeof a);
        const int nt = Bp / TILE_W;
        a.X = x.x, a.W0 = Wb[0], a.W1 = Wb[1], a.W1t = Wt[1];
        a.ldx = Kp[0], a.K0 = Kp[0];
        a.labels = labels, a.T = T, a.ldt = ldt, a.t_hi = 1.f, a.t_lo = t_lo;
        a.H0 = H[0], a.D2 = D[1], a.D1 = D[0], a.pbuf = wpbuf;
        a.cnt = wwords, a.flag = wwords + nt, a.err = wwords + 2 * nt;
        a.loss_acc = stats, a.correct = hits;
        a.Bp = Bp, a.n_valid = n_valid, a.n_out = n_out, a.type = type, a.ksplit = wide_ksplit;
        return hpnn_wide2_front(&a, s);
    }
    default: return -1;
    }
}

/* first-layer gradient slabs + the first [G1|G2] reduction pass (into midtmp) in one launch */
int BPlan::g0_reduce(const XIn &x, hipStream_t s) {
    const void *fm = fm_input(x);
    if (fm)
        return hpnn_gemm_fm_direct_reduce(D[0], fm, x.u8, x.u8 ? x.scale : 1.f, slab[0], Kp[0], Np[0], Kp[0], Bp, S[0],
                                          midslab, mid_grid, slab_f, slab_f, mid_groups, midtmp, s);
    if (mode == 't') return -2;
    return hpnn_gemm_tn_bf16_reduce(D[0], Np[0], x.x, Kp[0], slab[0], Kp[0], Np[0], Kp[0], Bp, S[0], midslab, mid_grid,
                                    slab_f, slab_f, mid_groups, midtmp, s);
}

/* G0 + its split-K reduction + every layer's step in ONE launch (kernels_g0.hip); -1 when
 * the shape or the input is not covered (the caller then runs G0 + the update launch) */
int BPlan::g0_fused_step(const XIn &x, float lr, float alpha, float scale, hipStream_t s, float *gout,
                         const unsigned int *gsel, long galt, const hpnn_xar_view *xv) {
    const void *fm = fm_input(x);
    if (!fm || !g0cnt || !g0_fused) return -1;
    hpnn_g0_update u;
    memset(&u, 0, sizeof u);
    u.gout = gout;
    u.gsel = gsel, u.galt = galt;
    if (xv) {
        /* HPNN_XAR_G0_MODE: 0 auto (two-shot from 4 ranks), 1 one-shot, 2 two-shot */
        static const int xm = [] { const char *e = getenv("HPNN_XAR_G0_MODE"); return e ? atoi(e) : 0; }();
        u.xchg = xm == 1 ? 1 : (xm == 2 || xv->world >= 4) ? 2 : 1;
        u.xv = *xv;
    }
    u.W32 = W32[0], u.V32 = V32[0], u.Wb = Wb[0], u.Wt = Wt[0], u.Wf = W0f;
    u.cnt = g0cnt, u.err = g0cnt + HPNN_G0_ERR_WORD;
    u.perm = g0_perm;
    if (g0_xcd && g0xw && g0xs) u.xw = g0xw, u.xslab = g0xs;
    u.fault = hpnn_fault_hit("handoff"); /* HPNN_FAULT=handoff:n: the n-th launch reports a timed-out wait */
    /* HPNN_FAULT=xsum:n: the n-th exchanging launch of the last rank sums one element wrong */
    u.xfault = xv && xv->world > 1 && xv->rank == xv->world - 1 && hpnn_fault_hit("xsum");
    u.lr = lr, u.alpha = alpha, u.scale = scale, u.momentum = momentum ? 1 : 0;
    u.mslab = midslab, u.mrows = mid_grid, u.mstride = slab_f, u.n12 = slab_f;
    for (int l = 0; l < 2; l++) {
        u.W32b[l] = W32[l + 1], u.V32b[l] = V32[l + 1], u.Wbb[l] = Wb[l + 1], u.Wtb[l] = Wt[l + 1];
        u.Nb[l] = Np[l + 1], u.Kb[l] = Kp[l + 1];
    }
    return hpnn_gemm_fm_direct_update(D[0], fm, x.u8, x.u8 ? x.scale : 1.f, slab[0], Kp[0], Np[0], Kp[0], Bp, S[0], &u,
                                      s);
}

/* the weight gradient and the step can run as ONE 8-phase TN launch (no gradient in memory):
 * one split, 256 x 256 tiles, no fragment-major W0 copy to keep (HPNN_TN_UPD=0: off) */
bool BPlan::tn_update_ok(int l) const {
    static const bool on = !env_off("HPNN_TN_UPD");
    return on && tn_update && l >= 0 && l < L && S[l] == 1 && Np[l] % 256 == 0 && Kp[l] % 256 == 0 && Bp % 128 == 0 && !(l == 0 && W0f);
}

/* from the last layer to the first: gradient + step per layer (the deltas were all computed
 * with the pre-update weights already) */
int BPlan::grad_and_update_layers(const XIn &x, float lr, float alpha, float scale, hipStream_t s) {
    /* a two-layer net (RRUFF): layer 1's gradient + step ride in layer 0's fused launch as its
     * side job (bitwise the separate gemm_tn + update launches; HPNN_TN8_SIDE=0: off) */
    if (L == 2 && tn8_side && tncnt && g0_fused && S[0] > 1 && !W0f) {
        hpnn_tn8_side sd = {D[1], H[0], Np[1], Kp[1], slab[1], Np[1], Kp[1], S[1],
                            W32[1], V32[1], Wb[1], Wt[1], tncnt + 1024 * L + 64};
        const int r = hpnn_gemm_tn8_fused_update_side(D[0], Np[0], x.x, Kp[0], Np[0], Kp[0], Bp, S[0], slab[0], W32[0],
                                                      V32[0], Wb[0], Wt[0], lr, alpha, scale, momentum ? 1 : 0, tncnt,
                                                      tncnt + 1024 * L, &sd, s);
        if (r == 0) {
            side_launches++;
            return 0;
        }
        if (r != -1 && r != -2) return r;
    }
    for (int l = L - 1; l >= 0; l--) {
        const void *Hin = l ? H[l - 1] : x.x;
        if (tn_update_ok(l) && hpnn_gemm_tn8_update(D[l], Np[l], Hin, Kp[l], Np[l], Kp[l], Bp, W32[l], V32[l], Wb[l],
                                                    Wt[l], lr, alpha, scale, momentum ? 1 : 0, s) == 0)
            continue;
        /* several splits: reduced and stepped inside the 8-phase TN launch (one layer at a
         * time: each layer has its own ticket block, every launch of it adds S[l] per tile) */
        if (tncnt && g0_fused && S[l] > 1 && !(l == 0 && W0f) &&
            hpnn_gemm_tn8_fused_update(D[l], Np[l], Hin, Kp[l], Np[l], Kp[l], Bp, S[l], slab[l], W32[l], V32[l], Wb[l],
                                       Wt[l], lr, alpha, scale, momentum ? 1 : 0, tncnt + 1024 * l, tncnt + 1024 * L,
                                       s) == 0)
            continue;
        int r = grad_layer(l, x, false, s);
        if (!r) r = update_layer(l, lr, alpha, scale, false, s);
        if (r) return r;
    }
    return 0;
}

int BPlan::step(const XIn &x, const int *labels, const float *T, int ldt, int n_valid, float lr, float alpha,
                hipStream_t s) {
    if (n_valid < 0 || n_valid > Bp) return -1;
    const float scale = 1.0f / (float)(n_valid > 0 ? n_valid : 1);
    int r;
    switch (mode) {
    case 't':
    case 'x':
    case 'm': {
        /* 3 launches: fused front; the G0 GEMM with the first [G1|G2] reduction pass on tail
         * workgroups appended to its grid (they fill the CUs the GEMM tiles leave idle); every
         * layer's update in one launch */
        if ((r = front(x, labels, T, ldt, n_valid, s))) return r;
        if ((r = g0_fused_step(x, lr, alpha, scale, s)) != -1) return r; /* 2 launches */
        if ((r = g0_reduce(x, s))) return r;
        const long n1 = (long)Np[1] * Kp[1];
        hpnn_upd_layer u[3] = {
            {W32[0], V32[0], slab[0], (long)Np[0] * Kp[0], Wb[0], Wt[0], W0f, S[0], Np[0], Kp[0]},
            {W32[1], V32[1], midtmp, slab_f, Wb[1], Wt[1], nullptr, mid_groups, Np[1], Kp[1]},
            {W32[2], V32[2], midtmp + n1, slab_f, Wb[2], Wt[2], nullptr, mid_groups, Np[2], Kp[2]}};
        return hpnn_sgd_update_multi(u, 3, lr, alpha, scale, momentum ? 1 : 0, s);
    }
    case 'w':
        /* one launch up to the deltas, then per-layer gradient + step (one multi-layer update
         * launch measured no faster: 22.1 vs 2 x 10.7 us) */
        if ((r = front(x, labels, T, ldt, n_valid, s))) return r;
        return grad_and_update_layers(x, lr, alpha, scale, s);
    default: {
        if ((r = forward(x.x, s))) return r;
        if ((r = output(labels, T, ldt, n_valid, nullptr, 0, true, s))) return r;
        for (int l = L - 1; l >= 1; l--)
            if ((r = backward_layer(l, s))) return r;
        /* every delta above used the pre-update weights: all gradients, then ONE update launch
         * for the layers whose step did not already run in the gradient GEMM's epilogue */
        hpnn_upd_layer u[HPNN_UPD_MAX];
        int nu = 0;
        for (int l = 0; l < L; l++) {
            const void *Hin = l ? H[l - 1] : x.x;
            if (tn_update_ok(l) && hpnn_gemm_tn8_update(D[l], Np[l], Hin, Kp[l], Np[l], Kp[l], Bp, W32[l], V32[l],
                                                        Wb[l], Wt[l], lr, alpha, scale, momentum ? 1 : 0, s) == 0)
                continue;
            if ((r = grad_layer(l, x, false, s))) return r;
            if (L <= HPNN_UPD_MAX)
                u[nu++] = {W32[l], V32[l], slab[l], (long)Np[l] * Kp[l], Wb[l], Wt[l], nullptr, S[l], Np[l], Kp[l]};
            else if ((r = update_layer(l, lr, alpha, scale, false, s)))
                return r;
        }
        return nu ? hpnn_sgd_update_multi(u, nu, lr, alpha, scale, momentum ? 1 : 0, s) : 0;
    }
    }
}

std::vector<std::pair<int, int>> BPlan::buckets() const {
    if (mode == 't' || mode == 'x' || mode == 'm') return {{1, 2}, {0, 0}};
    std::vector<std::pair<int, int>> v;
    for (int l = L - 1; l >= 0; l--) v.push_back({l, l});
    return v;
}

int BPlan::grads(const XIn &x, const int *labels, const float *T, int ldt, int n_valid, const ReadyFn &ready,
                 hipStream_t s) {
    int r;
    switch (mode) {
    case 't':
    case 'x':
    case 'm':
        if ((r = front(x, labels, T, ldt, n_valid, s))) return r;
        /* [G1 | G2] slab rows are exactly layers 1, 2 of the flat buffer: final first, so their
         * exchange overlaps the G0 GEMM */
        if ((r = hpnn_reduce_slabs2(midslab, mid_grid, slab_f, slab_f, midtmp, gflat + goff[1], s))) return r;
        if (!ready(1, 2)) return -8;
        if ((r = grad_layer(0, x, true, s))) return r;
        return ready(0, 0) ? 0 : -8;
    case 'w':
        if ((r = front(x, labels, T, ldt, n_valid, s))) return r;
        for (int l = 1; l >= 0; l--) {
            if ((r = grad_layer(l, x, true, s))) return r;
            if (!ready(l, l)) return -8;
        }
        return 0;
    default:
        if ((r = forward(x.x, s))) return r;
        if ((r = output(labels, T, ldt, n_valid, nullptr, 0, true, s))) return r;
        /* layer by layer from the top: the delta for layer l-1 (pre-update W_l), then layer l's
         * gradient into its bucket -- its exchange overlaps the layers below */
        for (int l = L - 1; l >= 0; l--) {
            if (l >= 1 && (r = backward_layer(l, s))) return r;
            if ((r = grad_layer(l, x, true, s))) return r;
            if (!ready(l, l)) return -8;
        }
        return 0;
    }
}

int BPlan::grads_local(const XIn &x, const int *labels, const float *T, int ldt, int n_valid, hipStream_t s) {
    if (mode != 't' && mode != 'x' && mode != 'm') return -1;
    int r;
    if ((r = front(x, labels, T, ldt, n_valid, s))) return r;
    if ((r = g0_fused_step(x, 0.f, 0.f, 0.f, s, gflat)) != -1) return r;
    /* not covered: slabs, then the reductions into the buffer */
    if ((r = g0_reduce(x, s))) return r;
    if ((r = hpnn_reduce_slabs(slab[0], S[0], (long)Np[0] * Kp[0], (long)Np[0] * Kp[0], gflat, s))) return r;
    return hpnn_reduce_slabs(midtmp, mid_groups, slab_f, slab_f, gflat + goff[1], s);
}

int BPlan::xchg_step(const XIn &x, const int *labels, const float *T, int ldt, int n_valid, float lr, float alpha,
                     float scale, const hpnn_xar_view &xv, hipStream_t s) {
    if (mode != 't' && mode != 'x' && mode != 'm') return -1;
    if (!fm_input(x) || !g0cnt || !g0_fused || !hpnn_gemm_fm_direct_update_ok(Kp[0], Np[0], Kp[0], Bp, S[0]) ||
        S[0] * hpnn_g0_tiles(x.u8, Np[0], Kp[0]) > HPNN_XAR_MAX_BLOCKS || (long)goff[L] > xv.half)
        return -1;
    int r;
    if ((r = front(x, labels, T, ldt, n_valid, s))) return r;
    r = g0_fused_step(x, lr, alpha, scale, s, nullptr, nullptr, 0, &xv);
    return r == -1 ? -9 : r; /* covered above: a refusal now is an error, not a fallback */
}

/* the in-kernel exchange on the real links before it carries a gradient: the fused G0 launch
 * in self-test mode (no GEMM) exchanges a known rank-dependent pattern over this communicator
 * and stores the rank-order sums in gflat; they must be exact.  Collective (every rank of the
 * view launches it); returns the number of wrong floats, < 0 on a launch / copy error, 1 when
 * the shape does not take the in-kernel exchange at all. */
int BPlan::xchg_self_test(const hpnn_xar_view &xv, hipStream_t s) {
    if (mode != 't' && mode != 'x' && mode != 'm') return -1;
    if (!g0cnt || !g0_fused || !hpnn_gemm_fm_direct_update_ok(Kp[0], Np[0], Kp[0], Bp, S[0]) ||
        S[0] * hpnn_g0_tiles(1, Np[0], Kp[0]) > HPNN_XAR_MAX_BLOCKS || (long)goff[L] > xv.half)
        return -1;
    hpnn_g0_update u;
    memset(&u, 0, sizeof u);
    u.xchg = 1;
    u.xv = xv;
    u.xtest = 1;
    u.xres = gflat;
    u.perm = g0_perm;
    u.W32 = W32[0], u.V32 = V32[0], u.Wb = Wb[0], u.Wt = Wt[0], u.Wf = W0f;
    u.cnt = g0cnt, u.err = g0cnt + HPNN_G0_ERR_WORD;
    u.momentum = momentum ? 1 : 0;
    u.mslab = midslab, u.mrows = mid_grid, u.mstride = slab_f, u.n12 = slab_f;
    for (int l = 0; l < 2; l++) {
        u.W32b[l] = W32[l + 1], u.V32b[l] = V32[l + 1], u.Wbb[l] = Wb[l + 1], u.Wtb[l] = Wt[l + 1];
        u.Nb[l] = Np[l + 1], u.Kb[l] = Kp[l + 1];
    }
    /* one-shot and two-shot both (the step picks by world size; HPNN_XAR_G0_MODE can force) */
    int bad = 0;
    const long n = goff[L];
    std::vector<float> h(n);
    for (int xm = 1; xm <= 2; xm++) {
        u.xchg = xm;
        if (hipMemsetAsync(gflat, 0xff, n * 4, s) != hipSuccess) return -3;
        const int r = hpnn_gemm_fm_direct_update(D[0], D[0], 1, 1.f, slab[0], Kp[0], Np[0], Kp[0], Bp, S[0], &u, s);
        if (r) return r < 0 ? r : -r;
        if (hipMemcpyAsync(h.data(), gflat, n * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return -3;
        const double tri = 0.5 * xv.world * (xv.world + 1);
        for (long i = 0; i < n; i++)
            if (h[i] != (float)(tri * ((i % 97) + 1) * 0.0625)) bad++;
    }
    return bad;
}

int BPlan::grads_slabs(const XIn &x, const int *labels, const float *T, int ldt, int n_valid, SlabSegs *segs,
                       hipStream_t s, float *dst, const unsigned int *sel, long alt) {
    if (mode != 't' && mode != 'x' && mode != 'm') return -1;
    int r;
    if ((r = front(x, labels, T, ldt, n_valid, s))) return r;
    if (dst && g0_fused_step(x, 0.f, 0.f, 0.f, s, dst, sel, alt) == 0) {
        segs->count = 0; /* already in the all-reduce's buffer */
        return 0;
    }
    if (!dst && g0_fused_step(x, 0.f, 0.f, 0.f, s, gflat) == 0) {
        /* G0 and [G1 | G2] reduced in the G0 launch: the exchange moves ONE copy */
        segs->count = 1;
        segs->base[0] = gflat;
        segs->cnt[0] = 1;
        segs->n[0] = segs->stride[0] = (long)goff[L];
        return 0;
    }
    if ((r = g0_reduce(x, s))) return r;
    segs->count = 2;
    segs->base[0] = slab[0];
    segs->cnt[0] = S[0];
    segs->n[0] = segs->stride[0] = (long)Np[0] * Kp[0];
    segs->base[1] = midtmp;
    segs->cnt[1] = mid_groups;
    segs->n[1] = segs->stride[1] = slab_f;
    return 0;
}

int BPlan::update_flat(const float *G, float lr, float alpha, float scale, hipStream_t s) {
    if (L > HPNN_UPD_MAX) {
        for (int l = 0; l < L; l++) {
            int r = hpnn_sgd_update(W32[l], V32[l], G + goff[l], 1, 0, Wb[l], Wt[l], Np[l], Kp[l], lr, alpha, scale,
                                    momentum ? 1 : 0, s);
            if (r) return r;
        }
        return 0;
    }
    hpnn_upd_layer u[HPNN_UPD_MAX];
    for (int l = 0; l < L; l++)
        u[l] = {W32[l], V32[l], G + goff[l], 0, Wb[l], Wt[l], l == 0 ? W0f : nullptr, 1, Np[l], Kp[l]};
    return hpnn_sgd_update_multi(u, L, lr, alpha, scale, momentum ? 1 : 0, s);
}

int BPlan::predict(const void *X, int n_valid, float *O, int ldo, hipStream_t s) {
    int r = forward(X, s);
    if (r) return r;
    return output(lab0, nullptr, 0, n_valid, O, ldo, false, s);
}

int BPlan::health_enqueue(hipStream_t s, unsigned int *dst) {
    if (g0cnt && hipMemcpyAsync(&dst[0], g0cnt + HPNN_G0_ERR_WORD, 4, hipMemcpyDeviceToHost, s) != hipSuccess) return -7;
    if (tncnt && hipMemcpyAsync(&dst[1], tncnt + 1024 * L, 4, hipMemcpyDeviceToHost, s) != hipSuccess) return -7;
    if (wwords && hipMemcpyAsync(&dst[2], wwords + 2 * (Bp / TILE_W), 4, hipMemcpyDeviceToHost, s) != hipSuccess)
        return -7;
    return 0;
}

int BPlan::health(hipStream_t s) {
    unsigned int e[3] = {0, 0, 0};
    if (health_enqueue(s, e) != 0 || hipStreamSynchronize(s) != hipSuccess) return -7;
    return (e[0] || e[1] || e[2]) ? -9 : 0;
}

int BPlan::weights_digest(int which, unsigned long long *out, hipStream_t s) {
    if (!digest_ && hpnn_dev_malloc((void **)&digest_, sizeof *digest_) != hipSuccess) return -7;
    if (hipMemsetAsync(digest_, 0, sizeof *digest_, s) != hipSuccess) return -7;
    long base = 0;
    for (int l = 0; l < L; l++) {
        const long n = (long)Np[l] * Kp[l];
        int r = 0;
        if (which & 1) {
            if (!r) r = hpnn_hash_words(Wb[l], n * 2, base, digest_, s);
            if (!r) r = hpnn_hash_words(Wt[l], n * 2, base + n / 2, digest_, s);
            base += n;
        }
        if ((which & 2) && !r) {
            r = hpnn_hash_words(W32[l], n * 4, base, digest_, s);
            base += n;
        }
        if (r) return r;
    }
    if (hipMemcpyAsync(out, digest_, sizeof *out, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return -7;
    return 0;
}

int BPlan::read_stats(double *loss, unsigned int *hits, hipStream_t s) {
    std::vector<float> h((size_t)HPNN_STAT_SLOTS * HPNN_STAT_STRIDE);
    if (hipMemcpyAsync(h.data(), stats, h.size() * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return -7;
    double l = 0.0;
    unsigned int c = 0;
    for (int i = 0; i < HPNN_STAT_SLOTS; i++) {
        l += h[(size_t)i * HPNN_STAT_STRIDE];
        unsigned int u;
        memcpy(&u, &h[(size_t)i * HPNN_STAT_STRIDE + 1], 4);
        c += u;
    }
    *loss = l;
    *hits = c;
    return 0;
}

}  // namespace hpnn
