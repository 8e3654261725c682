/*
 * libhpnn FP64 CPU engine -- the exact-semantics oracle.
 *
 * One generic implementation covers the three network types instead of the
 * reference's per-type x per-BLAS-flavour x per-MPI copies
 * (ann.c:892-2467, snn.c:79-1595):
 *   forward   h_l = f(W_l h_{l-1}),  f(x) = 2/(1+e^-x) - 1     (ann.c:883)
 *   output    ANN: f(z);  SNN: e^{z-1}/(TINY+sum e^{z-1}) (snn.c:280-335);
 *             LNN: z (linear output, declared but unimplemented upstream)
 *   error     ANN/LNN: 1/2 sum (t-o)^2 (ann.c:1246-1275);
 *             SNN: -(1/N) sum_{o>0} t log(o+TINY) (snn.c:447-477)
 *   deltas    all computed with pre-update weights (ann.c:1279-1592)
 *   BP        W += lr d (x) h            (ann.c:1596-1872)
 *   BPM       dW += lr d (x) h; W += dW; dW *= alpha   (ann.c:1943-2277)
 *   return    Ep(before) - Ep(after a second forward)  (ann.c:1862-1871)
 * OpenMP parallelises over neurons (rows); the loops are written so that
 * every output element is produced by one thread in a fixed order, hence
 * the result is bitwise independent of the thread count.
 */
#include <libhpnn/ann.h>
#include <math.h>
#include <string.h>
#include <omp.h>

#include "../core/runtime_internal.h"

extern "C" DOUBLE ann_act(DOUBLE x) { return 2.0 / (1.0 + exp(-1.0 * x)) - 1.0; }
extern "C" DOUBLE ann_dact(DOUBLE y) { return -0.5 * (y * y - 1.0); }

static inline int nthreads(void) { return _NN(return, omp_threads)(); }
/* fork/join costs microseconds: small layers (the online loop runs up to 10^5
 * iterations per sample) stay on one thread; per-row results are identical either way */
static inline bool par(unsigned long work) { return work >= 16384UL; }

/* y[N] = W[N x M] x[M] (+ optional activation) */
static void gemv_rows(const layer_ann *l, const DOUBLE *x, DOUBLE *y, bool act) {
    const UINT N = l->n_neurons, M = l->n_inputs;
#pragma omp parallel for if (par((unsigned long)N * M)) num_threads(nthreads()) schedule(static)
    for (long j = 0; j < (long)N; j++) {
        const DOUBLE *w = l->weights + _2D_IDX(M, j, 0);
        DOUBLE s = 0.0;
        for (UINT i = 0; i < M; i++) s += w[i] * x[i];
        y[j] = act ? ann_act(s) : s;
    }
}

extern "C" void hpnn_cpu_forward(kernel_ann *k, nn_type type) {
    const DOUBLE *x = k->in;
    for (UINT l = 0; l < k->n_hiddens; l++) {
        gemv_rows(&k->hiddens[l], x, k->hiddens[l].vec, true);
        x = k->hiddens[l].vec;
    }
    layer_ann *o = &k->output;
    if (type == NN_TYPE_ANN) {
        gemv_rows(o, x, o->vec, true);
    } else if (type == NN_TYPE_SNN) {
        gemv_rows(o, x, o->vec, false);
        DOUBLE dv = HPNN_TINY;
        for (UINT j = 0; j < o->n_neurons; j++) {
            o->vec[j] = exp(o->vec[j] - 1.0);
            dv += o->vec[j];
        }
        for (UINT j = 0; j < o->n_neurons; j++) o->vec[j] /= dv;
    } else {
        gemv_rows(o, x, o->vec, false);
    }
}

extern "C" void ann_kernel_run(kernel_ann *k) { hpnn_cpu_forward(k, NN_TYPE_ANN); }
extern "C" void snn_kernel_run(kernel_ann *k) { hpnn_cpu_forward(k, NN_TYPE_SNN); }
extern "C" void lnn_kernel_run(kernel_ann *k) { hpnn_cpu_forward(k, NN_TYPE_LNN); }

extern "C" DOUBLE hpnn_cpu_error(const kernel_ann *k, nn_type type, const DOUBLE *t) {
    const UINT N = k->n_outputs;
    const DOUBLE *o = k->output.vec;
    DOUBLE Ep = 0.0;
    if (type == NN_TYPE_SNN) {
        for (UINT i = 0; i < N; i++)
            if (o[i] > 0.) Ep += t[i] * log(o[i] + HPNN_TINY);
        Ep *= -1.0 / (DOUBLE)N;
    } else {
        for (UINT i = 0; i < N; i++) Ep += (t[i] - o[i]) * (t[i] - o[i]);
        Ep *= 0.5;
    }
    return Ep;
}

/* deltas: d[L] (output) ... d[0]; storage provided by caller */
static void compute_deltas(const kernel_ann *k, nn_type type, const DOUBLE *t, DOUBLE **d) {
    const UINT H = k->n_hiddens;
    const layer_ann *o = &k->output;
    for (UINT i = 0; i < o->n_neurons; i++) {
        const DOUBLE diff = t[i] - o->vec[i];
        d[H][i] = (type == NN_TYPE_ANN) ? diff * ann_dact(o->vec[i]) : diff;
    }
    /* hidden: d_l[m] = f'(h_l[m]) sum_n W_{l+1}[n][m] d_{l+1}[n] */
    for (long l = (long)H - 1; l >= 0; l--) {
        const layer_ann *up = (l == (long)H - 1) ? o : &k->hiddens[l + 1];
        const UINT N = up->n_neurons, M = up->n_inputs;
        const DOUBLE *dn = d[l + 1];
        const DOUBLE *h = k->hiddens[l].vec;
#pragma omp parallel for if (par((unsigned long)N * M)) num_threads(nthreads()) schedule(static)
        for (long m = 0; m < (long)M; m++) {
            DOUBLE s = 0.0;
            for (UINT n = 0; n < N; n++) s += up->weights[_2D_IDX(M, n, m)] * dn[n];
            d[l][m] = s * ann_dact(h[m]);
        }
    }
}

static void update_layer(layer_ann *l, const DOUBLE *d, const DOUBLE *h, DOUBLE lr, DOUBLE *dw,
                         DOUBLE alpha) {
    const UINT N = l->n_neurons, M = l->n_inputs;
#pragma omp parallel for if (par((unsigned long)N * M)) num_threads(nthreads()) schedule(static)
    for (long j = 0; j < (long)N; j++) {
        DOUBLE *w = l->weights + _2D_IDX(M, j, 0);
        if (dw) {
            DOUBLE *v = dw + _2D_IDX(M, j, 0);
            for (UINT i = 0; i < M; i++) {
                v[i] += lr * d[j] * h[i];
                w[i] += v[i];
                v[i] *= alpha;
            }
        } else {
            /* reference operand order: w += lr*d[j]*h[i] */
            for (UINT i = 0; i < M; i++) w[i] += lr * d[j] * h[i];
        }
    }
}

extern "C" DOUBLE hpnn_cpu_train_step(kernel_ann *k, nn_type type, const DOUBLE *t, DOUBLE lr,
                                      BOOL momentum, DOUBLE alpha) {
    const UINT H = k->n_hiddens;
    /* scratch: reuse one allocation per call pattern (the reference
     * allocated and freed every call, ann.c:1620-1624) */
    static thread_local DOUBLE *pool = NULL;
    static thread_local size_t pool_sz = 0;
    size_t need = k->n_outputs;
    for (UINT l = 0; l < H; l++) need += k->hiddens[l].n_neurons;
    if (need > pool_sz) {
        free(pool);
        pool = (DOUBLE *)malloc(need * sizeof(DOUBLE));
        pool_sz = need;
    }
    DOUBLE *dptr[64];
    DOUBLE **d = (H + 1 <= 64) ? dptr : (DOUBLE **)malloc((H + 1) * sizeof(DOUBLE *));
    size_t off = 0;
    for (UINT l = 0; l < H; l++) {
        d[l] = pool + off;
        off += k->hiddens[l].n_neurons;
    }
    d[H] = pool + off;

    const DOUBLE Ep = hpnn_cpu_error(k, type, t);
    compute_deltas(k, type, t, d);
    const bool m = momentum && k->dw;
    /* output, hidden descending, layer 0 (reference order; deltas are
     * precomputed so the order does not change the result) */
    update_layer(&k->output, d[H], H ? k->hiddens[H - 1].vec : k->in, lr, m ? k->dw[H] : NULL, alpha);
    for (long l = (long)H - 1; l >= 0; l--)
        update_layer(&k->hiddens[l], d[l], l ? k->hiddens[l - 1].vec : k->in, lr, m ? k->dw[l] : NULL,
                     alpha);
    hpnn_cpu_forward(k, type);
    const DOUBLE Epr = hpnn_cpu_error(k, type, t);
    if (d != dptr) free(d);
    return Ep - Epr;
}

extern "C" BOOL ann_momentum_init(kernel_ann *k) {
    if (!k) return FALSE;
    if (k->dw) return TRUE;
    k->dw = (DOUBLE **)calloc(k->n_hiddens + 1, sizeof(DOUBLE *));
    for (UINT l = 0; l < k->n_hiddens; l++)
        k->dw[l] = (DOUBLE *)calloc((size_t)k->hiddens[l].n_neurons * k->hiddens[l].n_inputs, sizeof(DOUBLE));
    k->dw[k->n_hiddens] = (DOUBLE *)calloc((size_t)k->output.n_neurons * k->output.n_inputs, sizeof(DOUBLE));
    return TRUE;
}

extern "C" void ann_raz_momentum(kernel_ann *k) {
    if (!k || !k->dw) return;
    for (UINT l = 0; l < k->n_hiddens; l++)
        memset(k->dw[l], 0, sizeof(DOUBLE) * (size_t)k->hiddens[l].n_neurons * k->hiddens[l].n_inputs);
    memset(k->dw[k->n_hiddens], 0, sizeof(DOUBLE) * (size_t)k->output.n_neurons * k->output.n_inputs);
}

extern "C" void ann_momentum_free(kernel_ann *k) {
    if (!k || !k->dw) return;
    for (UINT l = 0; l <= k->n_hiddens; l++) free(k->dw[l]);
    free(k->dw);
    k->dw = NULL;
}

static void argmax_target(const DOUBLE *o, const DOUBLE *t, UINT n, UINT *max_p, UINT *p_trg) {
    DOUBLE probe = -1.0;
    *max_p = 0;
    *p_trg = 0;
    for (UINT i = 0; i < n; i++) {
        if (probe < o[i]) {
            probe = o[i];
            *max_p = i;
        }
        if (t[i] == 1.0) *p_trg = i;
    }
}

extern "C" DOUBLE hpnn_cpu_train_sample(kernel_ann *k, nn_type type, nn_train train, const DOUBLE *in,
                                        const DOUBLE *out, DOUBLE lr, DOUBLE alpha, DOUBLE delta,
                                        UINT *n_iter, BOOL *ok, DOUBLE *init_err, BOOL *first_ok) {
    const bool mom = (train == NN_TRAIN_BPM);
    const UINT min_iter = mom ? MIN_BPM_ITER : MIN_BP_ITER;
    const UINT max_iter = mom ? MAX_BPM_ITER : MAX_BP_ITER;
    if (delta <= 0.) delta = mom ? DELTA_BPM : DELTA_BP;
    if (mom) {
        ann_momentum_init(k);
        ann_raz_momentum(k); /* momentum lifetime = one sample (ann.c:2386) */
    }
    memcpy(k->in, in, sizeof(DOUBLE) * k->n_inputs);
    hpnn_cpu_forward(k, type);
    DOUBLE dEp = hpnn_cpu_error(k, type, out);
    if (init_err) *init_err = dEp;
    UINT iter = 0;
    BOOL is_ok = FALSE;
    do {
        iter++;
        dEp = hpnn_cpu_train_step(k, type, out, lr, mom, alpha);
        UINT max_p, p_trg;
        argmax_target(k->output.vec, out, k->n_outputs, &max_p, &p_trg);
        is_ok = (max_p == p_trg);
        if (iter == 1 && first_ok) *first_ok = is_ok;
        if (iter > max_iter) break;
        is_ok = is_ok && (iter > min_iter);
    } while ((dEp > delta) || !is_ok);
    if (n_iter) *n_iter = iter;
    if (ok) *ok = is_ok;
    return dEp;
}

static DOUBLE train_logged(kernel_ann *k, nn_type type, nn_train tr, DOUBLE *in, DOUBLE *out,
                           DOUBLE lr, DOUBLE alpha, DOUBLE delta) {
    UINT it = 0;
    BOOL ok = FALSE, first = FALSE;
    DOUBLE e0 = 0.;
    DOUBLE r = hpnn_cpu_train_sample(k, type, tr, in, out, lr, alpha, delta, &it, &ok, &e0, &first);
    NN_COUT(stdout, " init=%15.10f", e0);
    NN_COUT(stdout, first ? " OK" : " NO");
    NN_COUT(stdout, " N_ITER=%8u", it);
    NN_COUT(stdout, " final=%15.10f", r);
    NN_COUT(stdout, ok ? " SUCCESS!\n" : " FAIL!\n");
    return r;
}

/* reference-compatible wrappers with the reference CPU learning rates */
extern "C" DOUBLE ann_train_BP(kernel_ann *k, DOUBLE *in, DOUBLE *out, DOUBLE delta) {
    return train_logged(k, NN_TYPE_ANN, NN_TRAIN_BP, in, out, BP_LEARN_RATE, 0., delta);
}
extern "C" DOUBLE ann_train_BPM(kernel_ann *k, DOUBLE *in, DOUBLE *out, DOUBLE alpha, DOUBLE delta) {
    return train_logged(k, NN_TYPE_ANN, NN_TRAIN_BPM, in, out, BPM_LEARN_RATE, alpha, delta);
}
extern "C" DOUBLE snn_train_BP(kernel_ann *k, DOUBLE *in, DOUBLE *out, DOUBLE delta) {
    (void)delta; /* reference ignores it (snn.c:1495) */
    return train_logged(k, NN_TYPE_SNN, NN_TRAIN_BP, in, out, GPU_LEARN_RATE, 0., DELTA_BP);
}
extern "C" DOUBLE snn_train_BPM(kernel_ann *k, DOUBLE *in, DOUBLE *out, DOUBLE alpha, DOUBLE delta) {
    return train_logged(k, NN_TYPE_SNN, NN_TRAIN_BPM, in, out, GPU_LEARN_RATE, alpha, delta);
}
