/*
 * libhpnn FP64 CPU batched engine: the oracle for minibatch semantics.
 *
 * Batched mode (new; the reference only trains online):
 *   for a minibatch of B samples, deltas are computed per sample exactly as
 *   in the online engine, the weight "gradient" is the mean
 *   G_l = (1/B) sum_b d_l^b (x) h_{l-1}^b, and the update reuses the
 *   reference rules with G in place of d (x) h:
 *     BP : W += lr G
 *     BPM: dW += lr G; W += dW; dW *= alpha    (momentum persists across
 *          minibatches; it is zeroed once at the start of training)
 *   With B = 1 one BP step equals one reference BP iteration.
 * Reductions run in a fixed order (sample index ascending) so results do
 * not depend on the OpenMP thread count.
 */
#include <libhpnn/ann.h>
#include <libhpnn/observe.h>
#include <math.h>
#include <string.h>
#include <chrono>
#include <vector>

#include "../core/runtime_internal.h"
#include "../gpu/engine.h"

static inline DOUBLE act(DOUBLE x) { return 2.0 / (1.0 + exp(-1.0 * x)) - 1.0; }
static inline DOUBLE dact(DOUBLE y) { return -0.5 * (y * y - 1.0); }

extern "C" DOUBLE hpnn_cpu_batched_step(kernel_ann *k, nn_type type, const DOUBLE *X, const DOUBLE *T,
                                        UINT B, DOUBLE lr, BOOL momentum, DOUBLE alpha, UINT *hits) {
    const UINT L = k->n_hiddens + 1;
    std::vector<const layer_ann *> layers(L);
    for (UINT l = 0; l + 1 < L; l++) layers[l] = &k->hiddens[l];
    layers[L - 1] = &k->output;
    /* activations A[l]: B x N_l ; A[-1] = X */
    std::vector<std::vector<DOUBLE>> A(L), D(L);
    for (UINT l = 0; l < L; l++) {
        A[l].assign((size_t)B * layers[l]->n_neurons, 0.0);
        D[l].assign((size_t)B * layers[l]->n_neurons, 0.0);
    }
    const UINT n_out = k->n_outputs;
    std::vector<DOUBLE> loss(B, 0.0);
    std::vector<unsigned char> hit(B, 0);
    const int nt = _NN(return, omp_threads)();
#pragma omp parallel for num_threads(nt) schedule(static)
    for (long b = 0; b < (long)B; b++) {
        const DOUBLE *x = X + (size_t)b * k->n_inputs;
        for (UINT l = 0; l < L; l++) {
            const layer_ann *ly = layers[l];
            DOUBLE *y = A[l].data() + (size_t)b * ly->n_neurons;
            const bool last = (l == L - 1);
            for (UINT j = 0; j < ly->n_neurons; j++) {
                const DOUBLE *w = ly->weights + _2D_IDX(ly->n_inputs, j, 0);
                DOUBLE s = 0.0;
                for (UINT i = 0; i < ly->n_inputs; i++) s += w[i] * x[i];
                y[j] = (!last || type == NN_TYPE_ANN) ? act(s) : s;
            }
            if (last && type == NN_TYPE_SNN) {
                DOUBLE dv = HPNN_TINY;
                for (UINT j = 0; j < ly->n_neurons; j++) {
                    y[j] = exp(y[j] - 1.0);
                    dv += y[j];
                }
                for (UINT j = 0; j < ly->n_neurons; j++) y[j] /= dv;
            }
            x = y;
        }
        /* loss + output delta */
        const DOUBLE *o = A[L - 1].data() + (size_t)b * n_out;
        const DOUBLE *t = T + (size_t)b * n_out;
        DOUBLE *d = D[L - 1].data() + (size_t)b * n_out;
        DOUBLE Ep = 0.0;
        if (type == NN_TYPE_SNN) {
            for (UINT i = 0; i < n_out; i++)
                if (o[i] > 0.) Ep += t[i] * log(o[i] + HPNN_TINY);
            Ep *= -1.0 / (DOUBLE)n_out;
        } else {
            for (UINT i = 0; i < n_out; i++) Ep += (t[i] - o[i]) * (t[i] - o[i]);
            Ep *= 0.5;
        }
        loss[b] = Ep;
        UINT g = 0, tr = 0; /* argmax hit (first maximum, as the GPU kernels) */
        for (UINT i = 1; i < n_out; i++) {
            if (o[i] > o[g]) g = i;
            if (t[i] > t[tr]) tr = i;
        }
        hit[b] = g == tr;
        for (UINT i = 0; i < n_out; i++) d[i] = (type == NN_TYPE_ANN) ? (t[i] - o[i]) * dact(o[i]) : (t[i] - o[i]);
        /* hidden deltas */
        for (long l = (long)L - 2; l >= 0; l--) {
            const layer_ann *up = layers[l + 1];
            const UINT N = up->n_neurons, M = up->n_inputs;
            const DOUBLE *dn = D[l + 1].data() + (size_t)b * N;
            const DOUBLE *h = A[l].data() + (size_t)b * M;
            DOUBLE *dl = D[l].data() + (size_t)b * M;
            for (UINT m = 0; m < M; m++) {
                DOUBLE s = 0.0;
                for (UINT n = 0; n < N; n++) s += up->weights[_2D_IDX(M, n, m)] * dn[n];
                dl[m] = s * dact(h[m]);
            }
        }
    }
    /* gradient + update per layer */
    const DOUBLE inv_b = 1.0 / (DOUBLE)B;
    const bool mom = momentum && k->dw;
    for (UINT l = 0; l < L; l++) {
        layer_ann *ly = (layer_ann *)layers[l];
        const UINT N = ly->n_neurons, M = ly->n_inputs;
        const DOUBLE *H = l ? A[l - 1].data() : X;
        const DOUBLE *Dl = D[l].data();
        DOUBLE *dw = mom ? k->dw[l] : NULL;
#pragma omp parallel for num_threads(nt) schedule(static)
        for (long j = 0; j < (long)N; j++) {
            DOUBLE *w = ly->weights + _2D_IDX(M, j, 0);
            for (UINT i = 0; i < M; i++) {
                DOUBLE g = 0.0;
                for (UINT b = 0; b < B; b++) g += Dl[(size_t)b * N + j] * H[(size_t)b * M + i];
                g *= inv_b;
                if (dw) {
                    DOUBLE *v = dw + _2D_IDX(M, j, 0);
                    v[i] += lr * g;
                    w[i] += v[i];
                    v[i] *= alpha;
                } else {
                    w[i] += lr * g;
                }
            }
        }
    }
    DOUBLE s = 0.0;
    UINT c = 0;
    for (UINT b = 0; b < B; b++) {
        s += loss[b];
        c += hit[b];
    }
    if (hits) *hits += c;
    return s * inv_b;
}

extern "C" BOOL hpnn_cpu_train_batched(kernel_ann *k, const DOUBLE *X, const DOUBLE *T, UINT n,
                                       const hpnn_batched_opts *o, hpnn_batched_stats *st) {
    if (!k || n == 0) return FALSE;
    const bool mom = o->train == NN_TRAIN_BPM;
    if (mom) {
        const bool keep = o->resume && k->dw;
        ann_momentum_init(k);
        if (!keep) ann_raz_momentum(k);
    }
    const UINT B = o->batch ? o->batch : 1;
    auto t0 = std::chrono::steady_clock::now();
    UINT64 samples = 0;
    DOUBLE last = 0.0;
    for (UINT e = 0; e < o->epochs; e++) {
        DOUBLE acc = 0.0;
        UINT nb = 0, hits = 0;
        for (UINT s = 0; s < n; s += B) {
            UINT b = (n - s < B) ? n - s : B;
            last = hpnn_cpu_batched_step(k, o->type, X + (size_t)s * k->n_inputs, T + (size_t)s * k->n_outputs, b,
                                         o->lr, mom, o->alpha, &hits);
            acc += last;
            nb++;
            samples += b;
        }
        if (st) st->epoch_loss = acc / (nb ? nb : 1);
        if (hpnn_metrics_active())
            hpnn_metrics_epoch("cpu", o->epoch0 + e + 1, acc / (nb ? nb : 1), hits, n,
                               std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(), samples);
    }
    auto t1 = std::chrono::steady_clock::now();
    if (st) {
        st->last_loss = last;
        st->samples = samples;
        st->seconds = std::chrono::duration<double>(t1 - t0).count();
        /* accuracy of the final weights on the training set */
        UINT correct = 0;
        for (UINT s = 0; s < n; s++) {
            memcpy(k->in, X + (size_t)s * k->n_inputs, sizeof(DOUBLE) * k->n_inputs);
            hpnn_cpu_forward(k, o->type);
            const DOUBLE *t = T + (size_t)s * k->n_outputs;
            UINT g = 0, tr = 0;
            for (UINT i = 1; i < k->n_outputs; i++)
                if (k->output.vec[i] > k->output.vec[g]) g = i;
            for (UINT i = 1; i < k->n_outputs; i++)
                if (t[i] > t[tr]) tr = i;
            correct += (g == tr);
        }
        st->correct = correct;
    }
    /* the momentum stays in k->dw: nn_dump_state saves it for an exact resume */
    return TRUE;
}
