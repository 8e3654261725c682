/*
 * libhpnn GPU engines -- host orchestration (HIP runtime, gfx950).
 *
 * Online engine: one persistent kernel per training sample (online.hip).
 * Batched engine: per minibatch
 *     forward   gemm_nt(act) per layer          (MFMA bf16)
 *     output    output_delta (act/softmax+loss+delta+accuracy)
 *     backward  gemm_nt(W^T, * f'(h)) per layer (MFMA bf16)
 *     gradient  gemm_tn split-K FP32 slabs      (MFMA bf16, tr-LDS reads)
 *     update    sgd_update (slab reduce + BP/BPM + BF16 W / W^T refresh)
 * All launches go to one HIP stream; nothing synchronises the host inside
 * an epoch (the reference synchronised every iteration).
 * Weights: host FP64 kernel_ann is the I/O master; the device keeps FP32
 * masters (batched) or FP64 (online) and syncs back lazily.
 */
#include <hip/hip_runtime_api.h>
#include <libhpnn/ann.h>
#include <dlfcn.h>
#include <libhpnn/comm.h>
#include <libhpnn/observe.h>
#include <libhpnn/devmem.h>
#include <libhpnn/bootstrap.h>
#include <libhpnn/xar.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <chrono>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <thread>
#include <vector>

#include "../core/runtime_internal.h"
#include "engine.h"
#include "kernels.h"
#include "bplan.h"
#include "../dist/dp_exchange.h"

#define HIPCHK(x)                                                                           \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            NN_ERROR(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            return FALSE;                                                                   \
        }                                                                                   \
    } while (0)

extern void (*hpnn_gpu_model_destroy_hook)(kernel_ann *);

namespace {

struct GpuModel {
    int dev = 0;
    int L = 0;
    double *W[16] = {0};
    double *dW[16] = {0};
    double *x = nullptr, *t = nullptr, *out = nullptr, *result = nullptr, *scratch = nullptr;
    double *xch = nullptr;     /* cooperative online kernel: exchange vectors + partials */
    unsigned int *ctl = nullptr;
    long xch_bytes = 0;
    bool device_newer = false; /* device weights not yet copied to host */
    bool host_newer = true;    /* host weights not yet uploaded         */
    /* online training over several devices (or virtual slots on one device): slot 0 is
     * this model, slots[s - 1] the others; each slot's W holds valid values only in the rows
     * its workgroups own (see hpnn_online_args); the exchange buffer and control words are
     * one fine-grained allocation on slot 0's device that every slot maps */
    std::vector<GpuModel *> slots;
    int n_slots = 1, sgrid = 0;
    int spd = 1; /* slots per device: S for virtual slots on device 0, else train_nn -S (capped) */
    bool sstream_owned = true; /* false: sstream is one of the runtime's -S streams */
    double *sxch = nullptr;
    unsigned int *sctl = nullptr;
    long sxch_bytes = 0;
    hipStream_t sstream = nullptr;
    /* a slot layout (S, spd) the cooperative kernel refused for this net: not retried */
    int coop_bad_S = 0, coop_bad_spd = 0;
    /* a grid barrier timed out mid-sample: the device rows are part-updated and
     * unrecoverable, so training stops (hpnn_gpu_failed) instead of going on from them */
    bool failed = false;
};

std::mutex g_mu;
std::set<kernel_ann *> g_models;

layer_ann *layer_of(kernel_ann *k, int l) { return l < (int)k->n_hiddens ? &k->hiddens[l] : &k->output; }

void free_model(GpuModel *g) {
    if (!g) return;
    for (GpuModel *s : g->slots) free_model(s);
    g->slots.clear();
    hipSetDevice(g->dev);
    if (g->sxch) hipFree(g->sxch);
    if (g->sctl) hipFree(g->sctl);
    if (g->sstream && g->sstream_owned) hipStreamDestroy(g->sstream);
    for (int l = 0; l < 16; l++) {
        if (g->W[l]) hpnn_dev_free(g->W[l]);
        if (g->dW[l]) hpnn_dev_free(g->dW[l]);
    }
    if (g->x) hpnn_dev_free(g->x);
    if (g->t) hpnn_dev_free(g->t);
    if (g->out) hpnn_dev_free(g->out);
    if (g->result) hpnn_dev_free(g->result);
    if (g->scratch) hpnn_dev_free(g->scratch);
    if (g->xch) hpnn_dev_free(g->xch);
    if (g->ctl) hpnn_dev_free(g->ctl);
    delete g;
}

void destroy_hook(kernel_ann *k) {
    std::lock_guard<std::mutex> lk(g_mu);
    free_model((GpuModel *)k->gpu);
    k->gpu = nullptr;
    g_models.erase(k);
}

void gather_host(kernel_ann *k);

/* keep_slots: the caller trains on the slots; otherwise slot 0's partial rows are made
 * whole first (the single-device paths read every row of W) */
BOOL ensure_model(kernel_ann *k, UINT gpu, bool keep_slots = false) {
    hpnn_gpu_model_destroy_hook = destroy_hook;
    GpuModel *g = (GpuModel *)k->gpu;
    if (g && !keep_slots && g->n_slots > 1 && g->device_newer) gather_host(k);
    const int L = (int)k->n_hiddens + 1;
    if (L > 16) {
        NN_ERROR(stderr, "GPU engine supports at most 15 hidden layers\n");
        return FALSE;
    }
    if (!g) {
        g = new GpuModel();
        g->dev = hpnn_rt_device(gpu);
        g->L = L;
        HIPCHK(hipSetDevice(g->dev));
        size_t vec = k->n_inputs;
        for (int l = 0; l < L; l++) {
            layer_ann *ly = layer_of(k, l);
            HIPCHK(hpnn_dev_malloc(&g->W[l], sizeof(double) * (size_t)ly->n_neurons * ly->n_inputs));
            vec += 3 * (size_t)ly->n_neurons;
        }
        HIPCHK(hpnn_dev_malloc(&g->x, sizeof(double) * k->n_inputs));
        HIPCHK(hpnn_dev_malloc(&g->t, sizeof(double) * k->n_outputs));
        HIPCHK(hpnn_dev_malloc(&g->out, sizeof(double) * k->n_outputs));
        HIPCHK(hpnn_dev_malloc(&g->result, sizeof(double) * 8));
        HIPCHK(hpnn_dev_malloc(&g->scratch, sizeof(double) * vec));
        k->gpu = g;
        std::lock_guard<std::mutex> lk(g_mu);
        g_models.insert(k);
    }
    HIPCHK(hipSetDevice(g->dev));
    if (g->host_newer && !(keep_slots && g->device_newer)) {
        for (int l = 0; l < L; l++) {
            layer_ann *ly = layer_of(k, l);
            HIPCHK(hipMemcpy(g->W[l], ly->weights, sizeof(double) * (size_t)ly->n_neurons * ly->n_inputs,
                             hipMemcpyHostToDevice));
        }
        g->host_newer = false;
        g->device_newer = false;
    }
    return TRUE;
}

/* momentum buffers of model g, zeroed on stream st (the stream its kernel runs on, so the
 * memset is ordered before the kernel's momentum writes) */
BOOL ensure_momentum(kernel_ann *k, GpuModel *g, hipStream_t st) {
    for (int l = 0; l < g->L; l++) {
        layer_ann *ly = layer_of(k, l);
        size_t n = (size_t)ly->n_neurons * ly->n_inputs;
        if (!g->dW[l]) HIPCHK(hpnn_dev_malloc(&g->dW[l], sizeof(double) * n));
        HIPCHK(hipMemsetAsync(g->dW[l], 0, sizeof(double) * n, st));
    }
    return TRUE;
}

void fill_args(kernel_ann *k, GpuModel *g, nn_type type, hpnn_online_args *a) {
    memset(a, 0, sizeof(*a));
    a->L = g->L;
    a->n_in = (int)k->n_inputs;
    for (int l = 0; l < g->L; l++) {
        layer_ann *ly = layer_of(k, l);
        a->N[l] = (int)ly->n_neurons;
        a->M[l] = (int)ly->n_inputs;
        a->W[l] = g->W[l];
        a->dW[l] = g->dW[l];
    }
    a->type = type == NN_TYPE_ANN ? 0 : (type == NN_TYPE_LNN ? 1 : 2);
    a->x = g->x;
    a->t = g->t;
    a->out = g->out;
    a->scratch = g->scratch;
    a->result = g->result;
    a->use_lds = hpnn_online_vec_bytes(a) <= 150 * 1024;
}

}  // namespace

void hpnn_rt_release_device_state(void) {
    std::lock_guard<std::mutex> lk(g_mu);
    for (kernel_ann *k : g_models) {
        GpuModel *g = (GpuModel *)k->gpu;
        /* keep the host master current before the device goes away */
        if (g && g->device_newer) gather_host(k);
        free_model(g);
        k->gpu = nullptr;
    }
    g_models.clear();
}

extern "C" BOOL hpnn_gpu_online_prepare(kernel_ann *k, UINT gpu) { return ensure_model(k, gpu); }

namespace {
void gather_host(kernel_ann *k) {
    GpuModel *g = (GpuModel *)k->gpu;
    hipSetDevice(g->dev);
    hipStreamSynchronize(hpnn_rt_stream(0, 0));
    for (int l = 0; l < g->L; l++) {
        layer_ann *ly = layer_of(k, l);
        hipMemcpy(ly->weights, g->W[l], sizeof(double) * (size_t)ly->n_neurons * ly->n_inputs, hipMemcpyDeviceToHost);
    }
    if (g->n_slots > 1) {
        /* every row from the slot whose workgroups own it: row j -> workgroup j % total */
        const int total = g->n_slots * g->sgrid;
        for (int s = 1; s < g->n_slots; s++) {
            GpuModel *m = g->slots[s - 1];
            hipSetDevice(m->dev);
            for (int l = 0; l < g->L; l++) {
                layer_ann *ly = layer_of(k, l);
                const size_t M = ly->n_inputs;
                std::vector<double> tmp((size_t)ly->n_neurons * M);
                hipMemcpy(tmp.data(), m->W[l], sizeof(double) * tmp.size(), hipMemcpyDeviceToHost);
                for (UINT j = 0; j < ly->n_neurons; j++)
                    if ((int)(j % total) / g->sgrid == s) memcpy(ly->weights + j * M, tmp.data() + j * M, 8 * M);
            }
        }
        hipSetDevice(g->dev);
        /* the single-device paths read slot 0's W: it must be whole again */
        g->host_newer = true;
    }
    g->device_newer = false;
}
}  // namespace

extern "C" void hpnn_gpu_sync_host(kernel_ann *k) {
    if (!k || !k->gpu || !((GpuModel *)k->gpu)->device_newer) return;
    gather_host(k);
}

extern "C" BOOL hpnn_gpu_failed(const kernel_ann *k) { return k && k->gpu && ((GpuModel *)k->gpu)->failed; }

extern "C" void hpnn_gpu_mark_host_dirty(kernel_ann *k) {
    if (!k || !k->gpu) return;
    ((GpuModel *)k->gpu)->host_newer = true;
}

/* the slot layout of the online engine (pure: unit-tested on the CPU through ctypes,
 * tests/test_capi_cpu.py): returns the slot count S and sets *spd (slots per device) */
extern "C" int hpnn_online_slot_plan(int n_gpu, int n_streams, int mem_model, int env_slots, int *spd) {
    if (env_slots > 1) { /* virtual slots on device 0: at most 2 run concurrently (hardware queues) */
        static bool warned = false;
        if (env_slots > 2 && !warned) {
            NN_WARN(stderr, "HPNN_ONLINE_SLOTS=%d: capped to 2 slots on one device\n", env_slots);
            warned = true;
        }
        *spd = env_slots > 2 ? 2 : env_slots;
        return *spd;
    }
    const int ng = (n_gpu > 1 && mem_model == (int)CUDA_MEM_P2P) ? n_gpu : 1;
    /* -S on ONE device is a no-op: two stream slots only split the same CUs finer and pay the
     * system-scope exchange (4096-4096-230 BPM: 2745 it/s on one slot vs 2618 with -S 2,
     * profiles/r4/a_online_engine.jsonl); HPNN_ONLINE_SLOTS still forces virtual slots (tests) */
    int ns = ng > 1 ? n_streams : 1;
    if (ns > 2) {
        static bool warned = false;
        if (!warned) NN_WARN(stderr, "online GPU engine: %d streams per GPU requested, 2 slots per GPU used\n", ns);
        warned = true;
        ns = 2;
    }
    *spd = ns > 1 ? ns : 1;
    return ng * *spd;
}

namespace {

/* the stream slot s runs on: the runtime's stream (s mod spd) of its device when train_nn -S
 * created that many (the reference's slice per stream, libhpnn.c:471-505), else its own */
void slot_stream(GpuModel *m, int s, int spd) {
    const nn_runtime *rt = hpnn_rt_get();
    const bool shared = spd > 1 && rt && (int)rt->cudas.cuda_n_streams >= spd;
    if (m->sstream && m->sstream_owned && !shared) return;
    if (m->sstream && m->sstream_owned) hipStreamDestroy(m->sstream);
    m->sstream = nullptr;
    m->sstream_owned = !shared;
    if (shared) m->sstream = hpnn_rt_stream((UINT)(s / spd), (UINT)(s % spd));
    else if (hipStreamCreateWithFlags(&m->sstream, hipStreamNonBlocking) != hipSuccess) m->sstream = nullptr;
}

/* slot models for online training over S slots, spd of them per device (S devices with
 * train_nn -G S; -G G -S 2: two slots per device; HPNN_ONLINE_SLOTS: S virtual slots on
 * device 0) */
BOOL ensure_slots(kernel_ann *k, int S, int spd) {
    GpuModel *g = (GpuModel *)k->gpu;
    if (g->n_slots == S && g->spd == spd) return TRUE;
    for (GpuModel *m : g->slots) free_model(m);
    g->slots.clear();
    g->n_slots = 1;
    g->sgrid = 0;
    if (S <= 1) return TRUE;
    for (int s = 1; s < S; s++) {
        GpuModel *m = new GpuModel();
        m->dev = hpnn_rt_device((UINT)(s / spd));
        m->L = g->L;
        g->slots.push_back(m);
        HIPCHK(hipSetDevice(m->dev));
        for (int l = 0; l < g->L; l++) {
            layer_ann *ly = layer_of(k, l);
            HIPCHK(hpnn_dev_malloc(&m->W[l], sizeof(double) * (size_t)ly->n_neurons * ly->n_inputs));
        }
        HIPCHK(hpnn_dev_malloc(&m->x, sizeof(double) * k->n_inputs));
        HIPCHK(hpnn_dev_malloc(&m->t, sizeof(double) * k->n_outputs));
        HIPCHK(hpnn_dev_malloc(&m->out, sizeof(double) * k->n_outputs));
        HIPCHK(hpnn_dev_malloc(&m->result, sizeof(double) * 8));
        HIPCHK(hpnn_dev_malloc(&m->scratch, sizeof(double) * 8));
        slot_stream(m, s, spd);
        if (!m->sstream) return FALSE;
    }
    HIPCHK(hipSetDevice(g->dev));
    slot_stream(g, 0, spd);
    if (!g->sstream) return FALSE;
    g->n_slots = S;
    g->sgrid = 0;
    g->spd = spd;
    g->host_newer = true; /* every slot takes the host weights */
    NN_OUT(stdout, "online GPU engine: rows over %d slots (%d per GPU, %s streams)\n", S, spd,
           g->sstream_owned ? "own" : "runtime");
    return TRUE;
}

BOOL upload_slots(kernel_ann *k) {
    GpuModel *g = (GpuModel *)k->gpu;
    for (GpuModel *m : g->slots) {
        HIPCHK(hipSetDevice(m->dev));
        for (int l = 0; l < g->L; l++) {
            layer_ann *ly = layer_of(k, l);
            HIPCHK(hipMemcpy(m->W[l], ly->weights, sizeof(double) * (size_t)ly->n_neurons * ly->n_inputs,
                             hipMemcpyHostToDevice));
        }
    }
    HIPCHK(hipSetDevice(g->dev));
    return TRUE;
}

/* One sample of the reference's online training on a cooperative grid spanning S slots
 * (the reference shards every layer's rows over n_gpu x n_streams, cuda_ann.cu:533-1275,
 * with hub copies and a device sync per layer; here one persistent kernel per device
 * exchanges the layer outputs and delta partials through fine-grained memory inside the
 * convergence loop).  Returns FALSE when the net does not suit the cooperative kernel. */
BOOL train_sample_slots(kernel_ann *k, nn_type type, nn_train train, const DOUBLE *in, const DOUBLE *out, DOUBLE lr,
                        DOUBLE alpha, DOUBLE delta, double res[5], bool *timed_out) {
    GpuModel *g = (GpuModel *)k->gpu;
    const int S = g->n_slots;
    const bool mom = train == NN_TRAIN_BPM;
    hpnn_online_args a0;
    fill_args(k, g, type, &a0);
    const int grid = hpnn_online_coop_grid_slots(&a0, S, 128 / g->spd);
    if (grid <= 0) return FALSE;
    const int total = grid * S;
    g->sgrid = grid; /* fixed for a net and S: the row ownership gather_host relies on */
    const long need = hpnn_online_coop_xch_bytes(&a0, total);
    HIPCHK(hipSetDevice(g->dev));
    if (need > g->sxch_bytes) {
        if (g->sxch) HIPCHK(hipFree(g->sxch));
        g->sxch = nullptr;
        HIPCHK(hipExtMallocWithFlags((void **)&g->sxch, (size_t)need, hipDeviceMallocUncached));
        g->sxch_bytes = need;
    }
    if (!g->sctl) HIPCHK(hipExtMallocWithFlags((void **)&g->sctl, HPNN_ONLINE_CTL_BYTES, hipDeviceMallocUncached));
    HIPCHK(hipMemset(g->sctl, 0, HPNN_ONLINE_CTL_BYTES));
    for (int s = 0; s < S; s++) {
        GpuModel *m = s ? g->slots[s - 1] : g;
        HIPCHK(hipSetDevice(m->dev));
        /* every slot (slot 0 included) zeroes its momentum on its own stream */
        if (mom && !ensure_momentum(k, m, m->sstream)) return FALSE;
        HIPCHK(hipMemcpyAsync(m->x, in, sizeof(double) * k->n_inputs, hipMemcpyHostToDevice, m->sstream));
        HIPCHK(hipMemcpyAsync(m->t, out, sizeof(double) * k->n_outputs, hipMemcpyHostToDevice, m->sstream));
    }
    /* every slot's copies are in place before any slot starts spinning on the others */
    for (int s = 0; s < S; s++) {
        GpuModel *m = s ? g->slots[s - 1] : g;
        HIPCHK(hipSetDevice(m->dev));
        HIPCHK(hipStreamSynchronize(m->sstream));
    }
    for (int s = 0; s < S; s++) {
        GpuModel *m = s ? g->slots[s - 1] : g;
        HIPCHK(hipSetDevice(m->dev));
        hpnn_online_args a;
        fill_args(k, m, type, &a);
        a.momentum = mom;
        a.lr = lr;
        a.alpha = alpha;
        a.delta = delta > 0 ? delta : (mom ? DELTA_BPM : DELTA_BP);
        a.min_iter = mom ? MIN_BPM_ITER : MIN_BP_ITER;
        a.max_iter = mom ? MAX_BPM_ITER : MAX_BP_ITER;
        a.forward_only = 0;
        a.xch = g->sxch;
        a.ctl = g->sctl;
        a.dev_slot = s;
        a.n_slots = S;
        if (hpnn_online_coop_launch(&a, grid, m->sstream) != 0) {
            NN_ERROR(stderr, "online kernel launch failed on slot %d\n", s);
            return FALSE;
        }
    }
    for (int s = S - 1; s >= 0; s--) {
        GpuModel *m = s ? g->slots[s - 1] : g;
        HIPCHK(hipSetDevice(m->dev));
        HIPCHK(hipStreamSynchronize(m->sstream));
    }
    HIPCHK(hipSetDevice(g->dev));
    HIPCHK(hipMemcpy(res, g->result, sizeof(double) * 5, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(k->output.vec, g->out, sizeof(double) * k->n_outputs, hipMemcpyDeviceToHost));
    unsigned int err = 0;
    HIPCHK(hipMemcpy(&err, (const char *)g->sctl + 128 * sizeof(unsigned int), sizeof err, hipMemcpyDeviceToHost));
    *timed_out = err != 0;
    return TRUE;
}

/* online slots: HPNN_ONLINE_SLOTS=S runs S virtual slots on device 0 (tests of the
 * device-spanning protocol on one GPU); else n_gpu x min(-S, 2) slots, the reference's
 * rows over n_gpu x n_streams (cuda_ann.cu:533-1275).  At most two slots share a device:
 * every slot's persistent launch needs a hardware queue of its own to run concurrently with
 * the others (a process gets GPU_MAX_HW_QUEUES = 4, one of them the null stream's), and more
 * slots on one device only split the same CUs finer.  Slots go on several devices only
 * with the P2P memory model: the exchange buffer and barrier words live on device 0 and the
 * other devices' kernels access them directly, which needs peer mappings (runtime.cpp's
 * probe can pick CMM / EXP on a partial topology). */
int online_slots(int *spd) {
    const nn_runtime *rt = hpnn_rt_get();
    const char *e = getenv("HPNN_ONLINE_SLOTS");
    return hpnn_online_slot_plan(rt ? (int)rt->cudas.n_gpu : 1, rt ? (int)rt->cudas.cuda_n_streams : 1,
                                 rt ? (int)rt->cudas.mem_model : (int)CUDA_MEM_NONE, e ? atoi(e) : 0, spd);
}

}  // namespace

extern "C" DOUBLE hpnn_gpu_train_sample(kernel_ann *k, nn_type type, nn_train train, const DOUBLE *in,
                                        const DOUBLE *out, DOUBLE lr, DOUBLE alpha, DOUBLE delta, UINT *n_iter,
                                        BOOL *ok, DOUBLE *init_err, BOOL *first_ok) {
    if (k->gpu && ((GpuModel *)k->gpu)->failed) {
        if (ok) *ok = FALSE;
        return 0.0;
    }
    {
        int spd = 1;
        const int S = online_slots(&spd);
        GpuModel *g0 = (GpuModel *)k->gpu;
        if (S > 1 && !(g0 && g0->coop_bad_S == S && g0->coop_bad_spd == spd)) {
            if (!k->gpu && !ensure_model(k, 0, true)) return 0.0;
            GpuModel *g = (GpuModel *)k->gpu;
            /* a different slot layout: the host takes the current rows first */
            if (g->device_newer && (g->n_slots != S || g->spd != spd)) gather_host(k);
            if (!ensure_slots(k, S, spd)) return 0.0;
            if (g->host_newer && !(ensure_model(k, 0, true) && upload_slots(k))) return 0.0;
            double res[5] = {0, 0, 0, 0, 0};
            bool to = false;
            if (train_sample_slots(k, type, train, in, out, lr, alpha, delta, res, &to)) {
                g->device_newer = true;
                if (to) {
                    NN_ERROR(stderr, "device-spanning online kernel: a grid barrier timed out; training stops\n");
                    g->failed = true;
                    g->device_newer = false; /* part-updated rows: never gathered into the host */
                    if (ok) *ok = FALSE;
                    return 0.0;
                }
                if (n_iter) *n_iter = (UINT)res[2];
                if (ok) *ok = res[3] != 0.0;
                if (init_err) *init_err = res[1];
                if (first_ok) *first_ok = res[4] != 0.0;
                return res[0];
            }
            /* the net does not suit the cooperative kernel: one device, and this layout is
             * not tried again for this model (no per-sample gather / slot re-allocation) */
            if (g->device_newer) gather_host(k);
            ensure_slots(k, 1, 1);
            g->coop_bad_S = S;
            g->coop_bad_spd = spd;
        }
    }
    if (!ensure_model(k, 0)) return 0.0;
    GpuModel *g = (GpuModel *)k->gpu;
    hipStream_t s = hpnn_rt_stream(0, 0);
    const bool mom = train == NN_TRAIN_BPM;
    if (mom && !ensure_momentum(k, g, s)) return 0.0; /* momentum reset per sample */
    hpnn_online_args a;
    fill_args(k, g, type, &a);
    a.momentum = mom;
    a.lr = lr;
    a.alpha = alpha;
    a.delta = delta > 0 ? delta : (mom ? DELTA_BPM : DELTA_BP);
    a.min_iter = mom ? MIN_BPM_ITER : MIN_BP_ITER;
    a.max_iter = mom ? MAX_BPM_ITER : MAX_BP_ITER;
    a.forward_only = 0;
    hipMemcpyAsync(g->x, in, sizeof(double) * k->n_inputs, hipMemcpyHostToDevice, s);
    hipMemcpyAsync(g->t, out, sizeof(double) * k->n_outputs, hipMemcpyHostToDevice, s);
    /* layers wide enough to spread over many CUs: the cooperative kernel (rows dealt to
     * resident workgroups), else the single-workgroup kernel */
    const int grid = hpnn_online_coop_grid(&a);
    if (grid > 0) {
        const long need = hpnn_online_coop_xch_bytes(&a, grid);
        if (need > g->xch_bytes) {
            if (g->xch) hpnn_dev_free(g->xch);
            g->xch = nullptr;
            g->xch_bytes = 0;
            if (hpnn_dev_malloc(&g->xch, (size_t)need) != hipSuccess) return 0.0;
            g->xch_bytes = need;
        }
        if (!g->ctl && hpnn_dev_malloc(&g->ctl, HPNN_ONLINE_CTL_BYTES) != hipSuccess) return 0.0;
        a.xch = g->xch;
        a.ctl = g->ctl;
    }
    if ((grid > 0 ? hpnn_online_coop_launch(&a, grid, s) : hpnn_online_launch(&a, s)) != 0) {
        NN_ERROR(stderr, "online kernel launch failed\n");
        return 0.0;
    }
    double res[5];
    hipMemcpyAsync(res, g->result, sizeof(res), hipMemcpyDeviceToHost, s);
    hipMemcpyAsync(k->output.vec, g->out, sizeof(double) * k->n_outputs, hipMemcpyDeviceToHost, s);
    hipStreamSynchronize(s);
    if (grid > 0 && hpnn_online_coop_status(&a) != 0) {
        NN_ERROR(stderr, "cooperative online kernel: a grid barrier timed out; training stops\n");
        g->failed = true;
        g->device_newer = false; /* part-updated rows: never gathered into the host */
        if (ok) *ok = FALSE;
        return 0.0;
    }
    g->device_newer = true;
    if (n_iter) *n_iter = (UINT)res[2];
    if (ok) *ok = res[3] != 0.0;
    if (init_err) *init_err = res[1];
    if (first_ok) *first_ok = res[4] != 0.0;
    return res[0];
}

extern "C" BOOL hpnn_gpu_forward(kernel_ann *k, nn_type type, const DOUBLE *in) {
    if (!ensure_model(k, 0)) return FALSE;
    GpuModel *g = (GpuModel *)k->gpu;
    hipStream_t s = hpnn_rt_stream(0, 0);
    hpnn_online_args a;
    fill_args(k, g, type, &a);
    a.forward_only = 1;
    hipMemcpyAsync(g->x, in, sizeof(double) * k->n_inputs, hipMemcpyHostToDevice, s);
    hipMemsetAsync(g->t, 0, sizeof(double) * k->n_outputs, s);
    if (hpnn_online_launch(&a, s) != 0) return FALSE;
    hipMemcpyAsync(k->output.vec, g->out, sizeof(double) * k->n_outputs, hipMemcpyDeviceToHost, s);
    memcpy(k->in, in, sizeof(double) * k->n_inputs);
    HIPCHK(hipStreamSynchronize(s));
    return TRUE;
}

/* ====================================================================== */
/* batched engine                                                          */
/* ====================================================================== */
namespace {

inline int pad_rows(int v, int m) { return (v + m - 1) / m * m; }

/* the resident training set on one device, in the layout the engine's kernels read: x =
 * the main input (row-major, or fragment-major for the tile front), xg = an optional
 * fragment-major 8-bit copy (first-layer gradient of mode 'x'); row r of a minibatch starts
 * r * row_bytes in (fragment-major layouts keep that for r % 32 == 0) */
struct XSet {
    void *x = nullptr, *xg = nullptr;
    int *lab = nullptr; /* class index per row when every target row is one-hot (else null) */
    size_t row_bytes = 0, row_bytes_g = 0;
    int u8 = 0;
    float scale = 1.f;
    void release() {
        hpnn_dev_free(x);
        hpnn_dev_free(xg);
        hpnn_dev_free(lab);
        x = xg = nullptr;
        lab = nullptr;
    }
};

/* one-hot targets (1 at the class, t_lo = 0 for SNN / -1 otherwise, every row of the set) ->
 * int32 class indices on the device (rows_p entries, 0 past n): the BF16 plan then takes the
 * label form of its output layer (no dense target rows to read).  FALSE only on a device
 * error; xs->lab stays null when the targets are not one-hot. */
BOOL attach_labels(XSet *xs, const DOUBLE *T, UINT n, int n_out, int rows_p, nn_type type, hipStream_t s) {
    const char *e = getenv("HPNN_LABELS");
    if (e && e[0] == '0') return TRUE;
    const DOUBLE t_lo = type == NN_TYPE_SNN ? 0.0 : -1.0;
    std::vector<int> lab((size_t)rows_p, 0);
    for (UINT i = 0; i < n; i++) {
        int c = -1;
        for (int j = 0; j < n_out; j++) {
            const DOUBLE t = T[(size_t)i * n_out + j];
            if (t == 1.0 && c < 0) c = j;
            else if (t != t_lo) return TRUE; /* dense targets */
        }
        if (c < 0) return TRUE;
        lab[i] = c;
    }
    if (hpnn_dev_malloc(&xs->lab, lab.size() * sizeof(int)) != hipSuccess) return FALSE;
    return hipMemcpyAsync(xs->lab, lab.data(), lab.size() * sizeof(int), hipMemcpyHostToDevice, s) == hipSuccess &&
           hipStreamSynchronize(s) == hipSuccess;
}

BOOL upload_bf16(const DOUBLE *src, int rows, int cols, int rows_p, int cols_p, void **dst, hipStream_t s);

/* round-to-nearest-even FP32 -> BF16 bits (the kernels' rounding) */
inline uint16_t bf16_bits(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return (uint16_t)((u + 0x7FFF + ((u >> 16) & 1)) >> 16);
}

/* host [rows][cols] -> fragment-major [rows_p/32][cols_p/16][64][8] (hpnn_amd.ops.to_fragment_major:
 * lane 16 g + r of fragment (t, cb) holds A[32 t + 8 g + j][16 cb + r], j < 8), zero padded */
template <typename E, typename Cvt>
std::vector<E> to_fragment_major(const DOUBLE *src, int rows, int cols, int rows_p, int cols_p, Cvt cvt) {
    std::vector<E> out((size_t)rows_p * cols_p, (E)0);
    const int nbc = cols_p / 16;
    for (int r = 0; r < rows; r++) {
        const int t = r / 32, g = (r % 32) / 8, j = r % 8;
        for (int c = 0; c < cols; c++) {
            const size_t idx = ((((size_t)t * nbc + c / 16) * 64) + 16 * g + c % 16) * 8 + j;
            out[idx] = cvt(src[(size_t)r * cols + c]);
        }
    }
    return out;
}

/* BF16 batched engine: an adapter of the library's batched plan (bplan.h, the same object
 * hpnn_amd.models.MLP binds) to the precision-generic drivers below */
struct Batched {
    typedef float target_t; /* dense targets, uploaded once */
    typedef float grad_t;   /* flat gradient buffer (the all-reduce payload) */
    static constexpr hpnn_comm_dtype comm_dt = HPNN_DT_F32;
    static const char *name() { return "bf16"; }
    static constexpr size_t ACC_BYTES = HPNN_STAT_SLOTS * HPNN_STAT_STRIDE * 4;
    static int reduce_sum(grad_t *buf, int G, size_t count, hipStream_t st) {
        return hpnn_reduce_slabs(buf, G, (long)count, (long)count, buf, st);
    }
    hpnn::BPlan p;
    int L = 0, Bp = 0;
    float *acc = nullptr, *gflat = nullptr;
    size_t goff[17] = {0};
    bool fm_ok = true; /* minibatch starts are multiples of 32 rows: fragment-major inputs */
    bool own_flat = false; /* the plan owns its flat buffer (loopback re-points it) */
    hipStream_t s = nullptr;

    ~Batched() {
        if (s) hipStreamSynchronize(s);
    }

    BOOL read_stats(double *loss, unsigned int *hits) { return p.read_stats(loss, hits, s) == 0; }

    /* allow_fm: every minibatch (shard) this net trains starts at a row multiple of 32;
     * fused: the plan's structure request (-1 auto, 0 per-layer only) */
    BOOL init(kernel_ann *k, int B, nn_type t, bool momentum, hipStream_t st, bool allow_fm = true, int fused = -1) {
        s = st;
        L = (int)k->n_hiddens + 1;
        std::vector<int> sizes(L + 1);
        sizes[0] = (int)k->n_inputs;
        for (int l = 0; l < L; l++) sizes[l + 1] = (int)layer_of(k, l)->n_neurons;
        const int type = t == NN_TYPE_ANN ? 0 : (t == NN_TYPE_LNN ? 1 : 2);
        std::string err;
        int rc = p.configure(sizes.data(), L, type, B, momentum, fused, nullptr, 512, true, &err);
        if (!rc && !allow_fm && p.mode == 't') /* the tile front reads fragment-major rows only */
            rc = p.configure(sizes.data(), L, type, B, momentum, 'x', nullptr, 512, true, &err);
        if (rc) {
            NN_ERROR(stderr, "batched plan: %s (%d)\n", err.c_str(), rc);
            return FALSE;
        }
        fm_ok = allow_fm;
        if (p.allocate(s)) return FALSE;
        Bp = p.Bp;
        for (int l = 0; l < L; l++) {
            layer_ann *ly = layer_of(k, l);
            const int M = (int)ly->n_inputs, N = (int)ly->n_neurons, Kp = p.Kp[l];
            std::vector<float> tmp((size_t)p.Np[l] * Kp, 0.f); /* FP64 host -> padded FP32 master */
            for (int n = 0; n < N; n++)
                for (int m = 0; m < M; m++) tmp[(size_t)n * Kp + m] = (float)ly->weights[(size_t)n * M + m];
            HIPCHK(hipMemcpyAsync(p.W32[l], tmp.data(), tmp.size() * 4, hipMemcpyHostToDevice, s));
            HIPCHK(hipStreamSynchronize(s));
        }
        if (p.cast_weights(s)) return FALSE;
        acc = p.stats;
        gflat = p.gflat;
        memcpy(goff, p.goff, sizeof goff);
        NN_DBG(stdout, "batched plan: mode %c, Bp %d, G0 splits %d\n", p.mode ? p.mode : '-', p.Bp, p.S[0]);
        return TRUE;
    }

    /* the training set in the plan's input layout: fragment-major for the tile front, plus a
     * fragment-major byte copy for mode 'x'; data that are all integers 0..255 (the reference's
     * pmnist pixels) go as bytes -- the same values, half the bytes of BF16 */
    BOOL upload_x(const DOUBLE *src, int rows, int cols, int rows_p, XSet *xs) {
        const int lay = fm_ok ? p.input_layout() : 0, Kp0 = p.Kp[0];
        rows_p = pad_rows(rows_p, 32);
        bool u8 = lay != 0;
        for (size_t i = 0; u8 && i < (size_t)rows * cols; i++) {
            const DOUBLE v = src[i];
            u8 = v >= 0.0 && v <= 255.0 && v == (DOUBLE)(int)v;
        }
        xs->u8 = u8 ? 1 : 0;
        xs->scale = 1.f;
        auto put = [&](const void *h, size_t bytes, void **dst) -> BOOL {
            HIPCHK(hpnn_dev_malloc(dst, bytes));
            HIPCHK(hipMemcpyAsync(*dst, h, bytes, hipMemcpyHostToDevice, s));
            HIPCHK(hipStreamSynchronize(s));
            return TRUE;
        };
        if (lay == 1) {
            if (u8) {
                auto h = to_fragment_major<uint8_t>(src, rows, cols, rows_p, Kp0, [](DOUBLE v) { return (uint8_t)v; });
                xs->row_bytes = Kp0;
                return put(h.data(), h.size(), &xs->x);
            }
            auto h = to_fragment_major<uint16_t>(src, rows, cols, rows_p, Kp0,
                                                 [](DOUBLE v) { return bf16_bits((float)v); });
            xs->row_bytes = (size_t)Kp0 * 2;
            return put(h.data(), h.size() * 2, &xs->x);
        }
        if (!upload_bf16(src, rows, cols, rows_p, Kp0, &xs->x, s)) return FALSE;
        xs->row_bytes = (size_t)Kp0 * 2;
        if (lay == 2 && u8) {
            auto h = to_fragment_major<uint8_t>(src, rows, cols, rows_p, Kp0, [](DOUBLE v) { return (uint8_t)v; });
            xs->row_bytes_g = Kp0;
            return put(h.data(), h.size(), &xs->xg);
        }
        xs->u8 = 0;
        return TRUE;
    }
    hpnn::XIn at(const XSet &xs, long row) const {
        hpnn::XIn v;
        v.x = (const char *)xs.x + row * xs.row_bytes;
        v.xg = xs.xg ? (const char *)xs.xg + row * xs.row_bytes_g : nullptr;
        v.u8 = xs.u8;
        v.scale = xs.scale;
        return v;
    }

    BOOL step(const XSet &xs, long row, const float *T, int ldt, int n_valid, float lr, float alpha, bool) {
        const int *L = xs.lab ? xs.lab + row : nullptr;
        const int r = p.step(at(xs, row), L, L ? nullptr : T, ldt, n_valid, lr, alpha, s);
        if (r) NN_ERROR(stderr, "batched step failed: %d\n", r);
        return r == 0 && hpnn_debug_check("batched training step") == 0;
    }

    /* data parallel: gradients into the flat FP32 buffer (the all-reduce payload) */
    BOOL alloc_flat(float *external = nullptr) {
        if (external) p.gflat = external; /* loopback: replicas' buffers in one allocation */
        gflat = p.gflat;
        return TRUE;
    }
    size_t flat_count() const { return p.goff[L]; }
    template <class Ready>
    BOOL grads(const XSet &xs, long row, const float *T, int ldt, int n_valid, Ready &&ready) {
        const int *L = xs.lab ? xs.lab + row : nullptr;
        const int r = p.grads(at(xs, row), L, L ? nullptr : T, ldt, n_valid, hpnn::ReadyFn(ready), s);
        if (r) NN_ERROR(stderr, "batched gradients failed: %d\n", r);
        return r == 0;
    }
    BOOL grads(const XSet &xs, long row, const float *T, int ldt, int n_valid) {
        /* no exchange to overlap (the xGMI all-reduce of the whole buffer follows): the fused
         * modes reduce G0 and [G1|G2] inside the G0 launch */
        const int *L = xs.lab ? xs.lab + row : nullptr;
        const int r = p.grads_local(at(xs, row), L, L ? nullptr : T, ldt, n_valid, s);
        if (r != -1) {
            if (r) NN_ERROR(stderr, "batched gradients failed: %d\n", r);
            return r == 0;
        }
        return grads(xs, row, T, ldt, n_valid, [](int, int) { return true; });
    }
    std::vector<std::pair<int, int>> buckets() const { return p.buckets(); }
    BOOL update_flat(const float *G, float lr, float alpha, float scale, bool) {
        return p.update_flat(G, lr, alpha, scale, s) == 0;
    }

    /* one process per GPU: the library's data-parallel step (dp_exchange.h) */
    std::unique_ptr<hpnn::DpExchange> dpx;
    bool attach_dpx(hpnn_comm *c, int mode) {
        dpx.reset(new hpnn::DpExchange());
        if (dpx->init(&p, c, mode)) dpx.reset();
        return (bool)dpx;
    }
    BOOL dp_step(const XSet &xs, long row, const float *T, int ldt, int nv, int total, float lr, float alpha) {
        const int *L = xs.lab ? xs.lab + row : nullptr;
        return dpx && dpx->step(at(xs, row), L, L ? nullptr : T, ldt, nv, total, lr, alpha, s) == 0;
    }
    BOOL gather_masters() { return !dpx || dpx->gather_masters(s) == 0; }
    /* fused modes: front + G0 with the exchange over xk and every layer's step in the same
     * launch (BPlan::xchg_step, the Python DataParallel's path); -1 = not covered */
    int xchg_step(const XSet &xs, long row, const float *T, int ldt, int nv, float lr, float alpha, float scale,
                  hpnn_xar *xk) {
        hpnn_xar_view v;
        if (hpnn_xar_view_get(xk, &v)) return -2;
        const int *L = xs.lab ? xs.lab + row : nullptr;
        return p.xchg_step(at(xs, row), L, L ? nullptr : T, ldt, nv, lr, alpha, scale, v, s);
    }
    bool has_dpx() const { return (bool)dpx; }
    void detach_dpx() { dpx.reset(); }

    /* FALSE when an in-kernel hand-off (fused G0 split-K tickets, fused TN tickets, the wide
     * front's tile pair) timed out since the plan was made: that launch stepped with partial
     * sums, so training must not go on from those weights (reference: CHK_ERR after every
     * launch, common.h:324-335) */
    BOOL healthy() {
        if (p.health(s) == 0) return TRUE;
        NN_ERROR(stderr, "batched GPU training: an in-kernel split-K / tile hand-off timed out "
                         "(the step used partial sums); stopping\n");
        return FALSE;
    }
    /* healthy() in two halves: enqueue the readback into d[0..2] (pinned, zeroed), judge it
     * once an event after it has completed */
    bool health_enqueue(unsigned int *d) { return p.health_enqueue(s, d) == 0; }
    BOOL health_ok(const unsigned int *d) {
        if (!(d[0] || d[1] || d[2])) return TRUE;
        NN_ERROR(stderr, "batched GPU training: an in-kernel split-K / tile hand-off timed out "
                         "(the step used partial sums); stopping\n");
        return FALSE;
    }
    /* digest of the weights every data-parallel replica must hold bit for bit: the BF16 copies,
     * plus the FP32 masters unless the BF16 reduce-scatter step keeps them sharded */
    BOOL digest(unsigned long long *d) {
        bool sh = false;
        for (int l = 0; dpx && l < L; l++) sh = sh || dpx->sharded(l);
        return p.weights_digest(sh ? 1 : 3, d, s) == 0;
    }

    /* FP32 master weights (and BPM momentum, into k->dw) -> host FP64 */
    BOOL download(kernel_ann *k) {
        HIPCHK(hipStreamSynchronize(s));
        if (p.V32[0]) ann_momentum_init(k);
        for (int l = 0; l < L; l++) {
            layer_ann *ly = layer_of(k, l);
            const int M = (int)ly->n_inputs, N = (int)ly->n_neurons, Kp = p.Kp[l];
            std::vector<float> tmp((size_t)p.Np[l] * Kp);
            HIPCHK(hipMemcpy(tmp.data(), p.W32[l], tmp.size() * 4, hipMemcpyDeviceToHost));
            for (int n = 0; n < N; n++)
                for (int m = 0; m < M; m++) ly->weights[(size_t)n * M + m] = tmp[(size_t)n * Kp + m];
            if (!p.V32[l]) continue;
            HIPCHK(hipMemcpy(tmp.data(), p.V32[l], tmp.size() * 4, hipMemcpyDeviceToHost));
            for (int n = 0; n < N; n++)
                for (int m = 0; m < M; m++) k->dw[l][(size_t)n * M + m] = tmp[(size_t)n * Kp + m];
        }
        return TRUE;
    }

    /* the replica state (FP32 masters + momentum, padded) as bytes, and back (then the BF16
     * copies are re-derived): rank 0's state re-broadcast after an exchange fallback */
    BOOL get_state(std::vector<char> &out) {
        out.clear();
        HIPCHK(hipStreamSynchronize(s));
        for (int l = 0; l < L; l++)
            for (float *b : {p.W32[l], p.V32[l]}) {
                if (!b) continue;
                const size_t n = (size_t)p.Np[l] * p.Kp[l] * 4, o = out.size();
                out.resize(o + n);
                HIPCHK(hipMemcpy(out.data() + o, b, n, hipMemcpyDeviceToHost));
            }
        return TRUE;
    }
    BOOL set_state(const char *in) {
        size_t o = 0;
        for (int l = 0; l < L; l++)
            for (float *b : {p.W32[l], p.V32[l]}) {
                if (!b) continue;
                const size_t n = (size_t)p.Np[l] * p.Kp[l] * 4;
                HIPCHK(hipMemcpy(b, in + o, n, hipMemcpyHostToDevice));
                o += n;
            }
        return p.cast_weights(s) == 0 && hipStreamSynchronize(s) == hipSuccess;
    }

    /* exact resume: BPM momentum k->dw (host FP64) -> padded FP32 V32 */
    BOOL upload_momentum(const kernel_ann *k) {
        if (!k->dw) return TRUE;
        for (int l = 0; l < L; l++) {
            if (!p.V32[l]) continue;
            const int M = (int)layer_of((kernel_ann *)k, l)->n_inputs, N = (int)layer_of((kernel_ann *)k, l)->n_neurons;
            const int Kp = p.Kp[l];
            std::vector<float> tmp((size_t)p.Np[l] * Kp, 0.f);
            for (int n = 0; n < N; n++)
                for (int m = 0; m < M; m++) tmp[(size_t)n * Kp + m] = (float)k->dw[l][(size_t)n * M + m];
            HIPCHK(hipMemcpyAsync(p.V32[l], tmp.data(), tmp.size() * 4, hipMemcpyHostToDevice, s));
            HIPCHK(hipStreamSynchronize(s));
        }
        return TRUE;
    }
};

/* upload n host rows (FP64) as a padded BF16 matrix [rows_p x cols_p] */
BOOL upload_bf16(const DOUBLE *src, int rows, int cols, int rows_p, int cols_p, void **dst, hipStream_t s) {
    void *tmp = nullptr;
    HIPCHK(hpnn_dev_malloc(dst, (size_t)rows_p * cols_p * 2));
    HIPCHK(hpnn_dev_malloc(&tmp, (size_t)rows * cols * 8));
    HIPCHK(hipMemcpyAsync(tmp, src, (size_t)rows * cols * 8, hipMemcpyHostToDevice, s));
    if (hpnn_pack_bf16(tmp, 1, rows, cols, cols, *dst, rows_p, cols_p, cols_p, s)) return FALSE;
    HIPCHK(hipStreamSynchronize(s));
    hpnn_dev_free(tmp);
    return TRUE;
}

/* FP64 / FP32 batched engine ([dtype] f64 | f32): the reference's precision (the
 * reference computes in double throughout, cuda_ann.cu:41-148, 546-548, 2139-2142) on the
 * FP64 / FP32 MFMA kernels of kernels_fp.hip.  Same minibatch semantics as the FP64 CPU
 * oracle (cpu_batched.cpp) and as Batched: forward, output delta, deltas with the
 * pre-update weights, G = sum over the batch, W updated with scale = 1 / n_valid.  No
 * padding: the kernels take any shape; the backward delta reads W itself (transposed
 * operand), so no W^T copy is kept. */
template <typename T>
struct BatchedFP {
    typedef T target_t;
    typedef T grad_t;
    static constexpr int F64 = sizeof(T) == 8 ? 1 : 0;
    static constexpr hpnn_comm_dtype comm_dt = sizeof(T) == 8 ? HPNN_DT_F64 : HPNN_DT_F32;
    static const char *name() { return sizeof(T) == 8 ? "f64" : "f32"; }
    static constexpr size_t ACC_BYTES = Batched::ACC_BYTES;
    int L = 0, Bp = 0, n_out = 0, type = 2;
    int M[16], N[16], S[16];
    int Kp[16]; /* Kp[0] = n_in: the row pitch of the uploaded input (drivers index rows by it) */
    T *W[16] = {0}, *V[16] = {0}, *slab[16] = {0}, *H[16] = {0}, *D[16] = {0};
    T *Z = nullptr, *gflat = nullptr;
    float *acc = nullptr;
    bool own_flat = false;
    size_t goff[17] = {0};
    hipStream_t s = nullptr;

    BOOL upload_x(const DOUBLE *src, int rows, int cols, int rows_p, XSet *xs) {
        std::vector<T> h((size_t)rows_p * cols, (T)0);
        for (size_t i = 0; i < (size_t)rows * cols; i++) h[i] = (T)src[i];
        HIPCHK(hpnn_dev_malloc(&xs->x, h.size() * sizeof(T)));
        HIPCHK(hipMemcpyAsync(xs->x, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice, s));
        HIPCHK(hipStreamSynchronize(s));
        xs->row_bytes = (size_t)cols * sizeof(T);
        return TRUE;
    }
    static const void *at(const XSet &xs, long row) { return (const char *)xs.x + row * xs.row_bytes; }
    static int reduce_sum(grad_t *buf, int G, size_t count, hipStream_t st) {
        return hpnn_reduce_fp(F64, buf, buf, G, (long)count, (long)count, st);
    }

    ~BatchedFP() {
        if (s) hipStreamSynchronize(s);
        if (dig) hpnn_dev_free(dig);
        for (int l = 0; l < 16; l++) {
            hpnn_dev_free(W[l]);
            hpnn_dev_free(V[l]);
            hpnn_dev_free(slab[l]);
            hpnn_dev_free(H[l]);
            hpnn_dev_free(D[l]);
        }
        hpnn_dev_free(Z);
        hpnn_dev_free(acc);
        if (own_flat) hpnn_dev_free(gflat);
    }

    BOOL read_stats(double *loss, unsigned int *hits) {
        std::vector<float> h(HPNN_STAT_SLOTS * HPNN_STAT_STRIDE);
        HIPCHK(hipMemcpyAsync(h.data(), acc, ACC_BYTES, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
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
        return TRUE;
    }

    /* split-K factor of a weight gradient over the batch: ~256 workgroups, >= 256 rows each */
    static int pick(int Nn, int Mm, int B) {
        const int tiles = ((Nn + 63) / 64) * ((Mm + 63) / 64);
        int sp = (256 + tiles - 1) / tiles;
        const int maxs = B / 256 > 0 ? B / 256 : 1;
        sp = sp < maxs ? sp : maxs;
        return hpnn_gemm_fp_splits(B, sp < 1 ? 1 : sp);
    }

    BOOL init(kernel_ann *k, int B, nn_type t, bool momentum, hipStream_t st, bool = true, int = -1) {
        s = st;
        L = (int)k->n_hiddens + 1;
        Bp = B;
        n_out = (int)k->n_outputs;
        type = t == NN_TYPE_ANN ? 0 : (t == NN_TYPE_LNN ? 1 : 2);
        for (int l = 0; l < L; l++) {
            layer_ann *ly = layer_of(k, l);
            M[l] = (int)ly->n_inputs;
            N[l] = (int)ly->n_neurons;
            Kp[l] = M[l];
            S[l] = pick(N[l], M[l], Bp);
            const size_t nw = (size_t)N[l] * M[l];
            HIPCHK(hpnn_dev_malloc(&W[l], nw * sizeof(T)));
            HIPCHK(hpnn_dev_malloc(&slab[l], nw * sizeof(T) * S[l]));
            if (momentum) {
                HIPCHK(hpnn_dev_malloc(&V[l], nw * sizeof(T)));
                HIPCHK(hipMemsetAsync(V[l], 0, nw * sizeof(T), s));
            }
            HIPCHK(hpnn_dev_malloc(&D[l], (size_t)Bp * N[l] * sizeof(T)));
            if (l < L - 1) HIPCHK(hpnn_dev_malloc(&H[l], (size_t)Bp * N[l] * sizeof(T)));
            std::vector<T> tmp(nw);
            for (size_t i = 0; i < nw; i++) tmp[i] = (T)ly->weights[i];
            HIPCHK(hipMemcpyAsync(W[l], tmp.data(), nw * sizeof(T), hipMemcpyHostToDevice, s));
            HIPCHK(hipStreamSynchronize(s));
        }
        HIPCHK(hpnn_dev_malloc(&Z, (size_t)Bp * N[L - 1] * sizeof(T)));
        HIPCHK(hpnn_dev_malloc(&acc, ACC_BYTES));
        HIPCHK(hipMemsetAsync(acc, 0, ACC_BYTES, s));
        return TRUE;
    }

    BOOL forward(const void *X, int rows) {
        for (int l = 0; l < L; l++) {
            const T *A = l ? H[l - 1] : (const T *)X;
            const bool last = l == L - 1;
            int r = hpnn_gemm_fp(F64, A, M[l], 0, W[l], M[l], 0, last ? (void *)Z : H[l], N[l], nullptr, 0, rows, N[l],
                                 M[l], last ? HPNN_EPI_NONE : HPNN_EPI_ACT, 1, 0, s);
            if (r) {
                NN_ERROR(stderr, "gemm_fp (fwd layer %d) failed: %d\n", l, r);
                return FALSE;
            }
        }
        return TRUE;
    }

    /* forward + output delta + hidden deltas + weight gradients (slab[l], S[l] slabs) */
    BOOL backprop(const void *X, const T *Tt, int ldt, int n_valid) {
        if (!forward(X, Bp)) return FALSE;
        if (hpnn_output_fp(F64, Z, N[L - 1], Tt, ldt, D[L - 1], N[L - 1], nullptr, 0, nullptr, acc,
                           (unsigned int *)(acc + 1), Bp, n_valid, n_out, type, s))
            return FALSE;
        for (int l = L - 1; l >= 1; l--) {
            /* D[l-1] = (D[l] W_l) * f'(H[l-1]): B(n = input m, k = neuron j) = W_l[j][m] */
            if (hpnn_gemm_fp(F64, D[l], N[l], 0, W[l], M[l], 1, D[l - 1], N[l - 1], H[l - 1], N[l - 1], Bp, M[l], N[l],
                             HPNN_EPI_DACT, 1, 0, s))
                return FALSE;
        }
        for (int l = 0; l < L; l++) {
            /* G[n][m] = sum_b D[b][n] H[b][m]: both operands transposed (k = the batch row) */
            const T *Hin = l ? H[l - 1] : (const T *)X;
            if (hpnn_gemm_fp(F64, D[l], N[l], 1, Hin, M[l], 1, slab[l], M[l], nullptr, 0, N[l], M[l], Bp,
                             HPNN_EPI_NONE, S[l], (long)N[l] * M[l], s))
                return FALSE;
        }
        return TRUE;
    }

    BOOL step(const XSet &xs, long row, const T *Tt, int ldt, int n_valid, double lr, double alpha, bool mom) {
        if (!backprop(at(xs, row), Tt, ldt, n_valid)) return FALSE;
        const double scale = 1.0 / (double)n_valid;
        for (int l = 0; l < L; l++)
            if (hpnn_update_fp(F64, W[l], V[l], slab[l], S[l], (long)N[l] * M[l], (long)N[l] * M[l], lr, alpha, scale,
                               mom ? 1 : 0, s))
                return FALSE;
        return hpnn_debug_check("batched training step (fp)") == 0;
    }

    BOOL alloc_flat(T *external = nullptr) {
        goff[0] = 0;
        for (int l = 0; l < L; l++) goff[l + 1] = goff[l] + (size_t)N[l] * M[l];
        if (external) {
            gflat = external;
            own_flat = false;
            return TRUE;
        }
        HIPCHK(hpnn_dev_malloc(&gflat, goff[L] * sizeof(T)));
        own_flat = true;
        return TRUE;
    }
    size_t flat_count() const { return goff[L]; }

    template <class Ready>
    BOOL grads(const XSet &xs, long row, const T *Tt, int ldt, int n_valid, Ready &&ready) {
        const void *X = at(xs, row);
        if (!forward(X, Bp)) return FALSE;
        if (hpnn_output_fp(F64, Z, N[L - 1], Tt, ldt, D[L - 1], N[L - 1], nullptr, 0, nullptr, acc,
                           (unsigned int *)(acc + 1), Bp, n_valid, n_out, type, s))
            return FALSE;
        for (int l = L - 1; l >= 0; l--) {
            if (l >= 1 && hpnn_gemm_fp(F64, D[l], N[l], 0, W[l], M[l], 1, D[l - 1], N[l - 1], H[l - 1], N[l - 1], Bp,
                                       M[l], N[l], HPNN_EPI_DACT, 1, 0, s))
                return FALSE;
            const T *Hin = l ? H[l - 1] : (const T *)X;
            if (hpnn_gemm_fp(F64, D[l], N[l], 1, Hin, M[l], 1, slab[l], M[l], nullptr, 0, N[l], M[l], Bp,
                             HPNN_EPI_NONE, S[l], (long)N[l] * M[l], s) ||
                hpnn_reduce_fp(F64, gflat + goff[l], slab[l], S[l], (long)N[l] * M[l], (long)N[l] * M[l], s))
                return FALSE;
            if (!ready(l, l)) return FALSE;
        }
        return TRUE;
    }
    BOOL grads(const XSet &xs, long row, const T *Tt, int ldt, int n_valid) {
        return grads(xs, row, Tt, ldt, n_valid, [](int, int) { return true; });
    }
    std::vector<std::pair<int, int>> buckets() const {
        std::vector<std::pair<int, int>> v;
        for (int l = L - 1; l >= 0; l--) v.push_back({l, l});
        return v;
    }

    BOOL update_flat(const T *G, double lr, double alpha, double scale, bool mom) {
        for (int l = 0; l < L; l++)
            if (hpnn_update_fp(F64, W[l], V[l], G + goff[l], 1, 0, (long)N[l] * M[l], lr, alpha, scale, mom ? 1 : 0, s))
                return FALSE;
        return TRUE;
    }

    bool attach_dpx(hpnn_comm *, int) { return false; } /* FP32 / FP64: the generic bucket loop */
    BOOL dp_step(const XSet &, long, const T *, int, int, int, double, double) { return FALSE; }
    int xchg_step(const XSet &, long, const T *, int, int, double, double, double, hpnn_xar *) { return -1; }
    BOOL gather_masters() { return TRUE; }
    BOOL healthy() { return TRUE; } /* no in-kernel hand-offs in the FP64 / FP32 kernels */
    bool health_enqueue(unsigned int *) { return true; }
    BOOL health_ok(const unsigned int *) { return TRUE; }
    unsigned long long *dig = nullptr; /* device word of digest() */
    BOOL digest(unsigned long long *d) {
        if (!dig && hpnn_dev_malloc((void **)&dig, 8) != hipSuccess) return FALSE;
        if (hipMemsetAsync(dig, 0, 8, s) != hipSuccess) return FALSE;
        long base = 0;
        for (int l = 0; l < L; l++) {
            const long nb = (long)N[l] * M[l] * (long)sizeof(T);
            if (hpnn_hash_words(W[l], nb, base, dig, s) != 0) return FALSE;
            base += nb / 4;
        }
        return hipMemcpyAsync(d, dig, 8, hipMemcpyDeviceToHost, s) == hipSuccess && hipStreamSynchronize(s) == hipSuccess;
    }
    bool has_dpx() const { return false; }
    void detach_dpx() {}

    BOOL download(kernel_ann *k) {
        HIPCHK(hipStreamSynchronize(s));
        if (V[0]) ann_momentum_init(k);
        for (int l = 0; l < L; l++) {
            layer_ann *ly = layer_of(k, l);
            const size_t nw = (size_t)N[l] * M[l];
            std::vector<T> tmp(nw);
            HIPCHK(hipMemcpy(tmp.data(), W[l], nw * sizeof(T), hipMemcpyDeviceToHost));
            for (size_t i = 0; i < nw; i++) ly->weights[i] = (DOUBLE)tmp[i];
            if (!V[l]) continue;
            HIPCHK(hipMemcpy(tmp.data(), V[l], nw * sizeof(T), hipMemcpyDeviceToHost));
            for (size_t i = 0; i < nw; i++) k->dw[l][i] = (DOUBLE)tmp[i];
        }
        return TRUE;
    }

    BOOL get_state(std::vector<char> &out) {
        out.clear();
        HIPCHK(hipStreamSynchronize(s));
        for (int l = 0; l < L; l++)
            for (T *b : {W[l], V[l]}) {
                if (!b) continue;
                const size_t n = (size_t)N[l] * M[l] * sizeof(T), o = out.size();
                out.resize(o + n);
                HIPCHK(hipMemcpy(out.data() + o, b, n, hipMemcpyDeviceToHost));
            }
        return TRUE;
    }
    BOOL set_state(const char *in) {
        size_t o = 0;
        for (int l = 0; l < L; l++)
            for (T *b : {W[l], V[l]}) {
                if (!b) continue;
                const size_t n = (size_t)N[l] * M[l] * sizeof(T);
                HIPCHK(hipMemcpy(b, in + o, n, hipMemcpyHostToDevice));
                o += n;
            }
        return TRUE;
    }

    BOOL upload_momentum(const kernel_ann *k) {
        if (!k->dw) return TRUE;
        for (int l = 0; l < L; l++) {
            if (!V[l]) continue;
            const size_t nw = (size_t)N[l] * M[l];
            std::vector<T> tmp(nw);
            for (size_t i = 0; i < nw; i++) tmp[i] = (T)k->dw[l][i];
            HIPCHK(hipMemcpyAsync(V[l], tmp.data(), nw * sizeof(T), hipMemcpyHostToDevice, s));
            HIPCHK(hipStreamSynchronize(s));
        }
        return TRUE;
    }
};

}  // namespace

namespace {

/* Data-parallel batched training driven by ONE process over G replicas (the reference's
 * single-process multi-GPU design, libhpnn.c:201-305, with its hub copies replaced by an
 * RCCL all-reduce over xGMI): every global minibatch of B samples is split into G shards
 * of ceil(B/G); each replica computes the gradient sum of its shard into a flat FP32
 * buffer; one grouped ncclAllReduce sums them; every replica applies the identical update
 * with scale 1/(samples of the minibatch), so the weights stay replicated and the result
 * equals the single-GPU step up to summation order.
 * loopback: G virtual replicas on ONE device (CI without a multi-GPU node): the buffers
 * live in one allocation and the all-reduce is a deterministic slab sum. */
template <class Net>
BOOL train_dp(kernel_ann *k, const DOUBLE *X, const DOUBLE *T, UINT n, const hpnn_batched_opts *o,
              hpnn_batched_stats *st, int G, bool loopback);
template <class Net>
BOOL train_dp_mp(kernel_ann *k, const DOUBLE *X, const DOUBLE *T, UINT n, const hpnn_batched_opts *o,
                 hpnn_batched_stats *st);
template <class Net>
BOOL train_single(kernel_ann *k, const DOUBLE *X, const DOUBLE *T, UINT n, const hpnn_batched_opts *o,
                  hpnn_batched_stats *st);

}  // namespace

extern "C" BOOL hpnn_gpu_train_batched(kernel_ann *k, const DOUBLE *X, const DOUBLE *T, UINT n,
                                       const hpnn_batched_opts *o, hpnn_batched_stats *st) {
    if (o->dtype != NN_DTYPE_BF16 && o->dtype != NN_DTYPE_F32 && o->dtype != NN_DTYPE_F64) {
        NN_ERROR(stderr, "GPU batched engine: unsupported dtype %d\n", (int)o->dtype);
        return FALSE;
    }
    if (o->tp) return hpnn_gpu_train_tp(k, X, T, n, o, st);
    const char *lb = getenv("HPNN_LOOPBACK_RANKS");
    const int lbr = lb ? atoi(lb) : 0;
    const char *fr = getenv("HPNN_FORCE_RCCL");
    const char *nd = getenv("HPNN_NATIVE_DP");
    const nn_dtype dt = o->dtype;
    if (lbr >= 2) {
        if (dt == NN_DTYPE_BF16) return train_dp<Batched>(k, X, T, n, o, st, lbr, true);
        if (dt == NN_DTYPE_F32) return train_dp<BatchedFP<float>>(k, X, T, n, o, st, lbr, true);
        return train_dp<BatchedFP<double>>(k, X, T, n, o, st, lbr, true);
    }
    /* one process per GPU under a launcher (torchrun --no-python bin/train_nn ...);
     * HPNN_DP_FORCE=1: the same path with ONE rank under a launcher (its step structure and
     * exchange kernels timed on a single GPU, as bench.py's HPNN_DP_FORCE) */
    const char *dpf = getenv("HPNN_DP_FORCE");
    const bool dp_one = dpf && dpf[0] == '1' && getenv("LOCAL_WORLD_SIZE") && hpnn_boot_world() == 1;
    if ((hpnn_boot_world() > 1 || dp_one) && !(nd && nd[0] == '0')) {
        if (dt == NN_DTYPE_BF16) return train_dp_mp<Batched>(k, X, T, n, o, st);
        if (dt == NN_DTYPE_F32) return train_dp_mp<BatchedFP<float>>(k, X, T, n, o, st);
        return train_dp_mp<BatchedFP<double>>(k, X, T, n, o, st);
    }
    if (o->n_gpu > 1 || (fr && fr[0] == '1')) {
        const int G = (int)(o->n_gpu ? o->n_gpu : 1);
        if (dt == NN_DTYPE_BF16) return train_dp<Batched>(k, X, T, n, o, st, G, false);
        if (dt == NN_DTYPE_F32) return train_dp<BatchedFP<float>>(k, X, T, n, o, st, G, false);
        return train_dp<BatchedFP<double>>(k, X, T, n, o, st, G, false);
    }
    if (dt == NN_DTYPE_BF16) return train_single<Batched>(k, X, T, n, o, st);
    if (dt == NN_DTYPE_F32) return train_single<BatchedFP<float>>(k, X, T, n, o, st);
    return train_single<BatchedFP<double>>(k, X, T, n, o, st);
}

namespace {

/* HIP graph of one epoch's steps (HPNN_GRAPH=0: eager launches): the epoch's minibatches
 * are the same every epoch (the sample order is drawn once, libhpnn.c:1218-1229), so one
 * capture is replayed per epoch and the host launches nothing per step.  Returns FALSE when
 * the launches cannot be captured (the caller then runs them eagerly: nothing of a failed
 * capture was executed). */
template <class Launch>
bool capture_epoch(hipStream_t s, Launch &&launch, hipGraphExec_t *exec) {
    *exec = nullptr;
    hipGraph_t g = nullptr;
    if (hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed) != hipSuccess) return false;
    const bool ok = launch();
    const hipError_t e = hipStreamEndCapture(s, &g);
    if (!ok || e != hipSuccess || !g) {
        if (g) hipGraphDestroy(g);
        hipGetLastError();
        return false;
    }
    const bool inst = hipGraphInstantiate(exec, g, nullptr, nullptr, 0) == hipSuccess;
    hipGraphDestroy(g);
    if (!inst) {
        *exec = nullptr;
        hipGetLastError();
    }
    return inst;
}

bool graphs_enabled() {
    const char *e = getenv("HPNN_GRAPH");
    return !(e && e[0] == '0') && !hpnn_debug_enabled();
}

template <class Net>
BOOL train_single(kernel_ann *k, const DOUBLE *X, const DOUBLE *T, UINT n, const hpnn_batched_opts *o,
                  hpnn_batched_stats *st) {
    typedef typename Net::target_t TT;
    if (k->n_hiddens + 1 > 16) return FALSE;
    hpnn_gpu_sync_host(k);
    HIPCHK(hipSetDevice(hpnn_rt_device(0)));
    hipStream_t s = hpnn_rt_stream(0, 0);
    const int B = (int)(o->batch ? o->batch : 256);
    const bool mom = o->train == NN_TRAIN_BPM;
    Net net;
    if (!net.init(k, B, o->type, mom, s, B % 32 == 0)) return FALSE;
    NN_OUT(stdout, "batched GPU training: %s, %d samples per step\n", Net::name(), B);
    if (mom && o->resume && !net.upload_momentum(k)) return FALSE;
    const int n_batches = (int)((n + B - 1) / B);
    const int rows_p = (n_batches - 1) * B + net.Bp; /* last batch reads Bp rows */
    XSet xs;
    TT *Td = nullptr;
    if (!net.upload_x(X, (int)n, (int)k->n_inputs, rows_p, &xs)) return FALSE;
    if (!attach_labels(&xs, T, n, (int)k->n_outputs, rows_p, o->type, s)) return FALSE;
    {
        std::vector<TT> tf((size_t)rows_p * k->n_outputs, (TT)0);
        for (size_t i = 0; i < (size_t)n * k->n_outputs; i++) tf[i] = (TT)T[i];
        HIPCHK(hpnn_dev_malloc(&Td, tf.size() * sizeof(TT)));
        HIPCHK(hipMemcpy(Td, tf.data(), tf.size() * sizeof(TT), hipMemcpyHostToDevice));
    }
    auto epoch = [&]() -> bool {
        for (int b = 0; b < n_batches; b++) {
            const int nv = (b == n_batches - 1) ? (int)n - b * B : B;
            if (!net.step(xs, (long)b * B, Td + (size_t)b * B * k->n_outputs, (int)k->n_outputs, nv, o->lr, o->alpha,
                          mom))
                return false;
        }
        return true;
    };
    /* ne epochs back to back; the statistics are zeroed before the last (the only one read) */
    auto epochs = [&](int ne) -> bool {
        for (int i = 0; i < ne; i++)
            if ((i + 1 == ne && hipMemsetAsync(net.acc, 0, Net::ACC_BYTES, s) != hipSuccess) || !epoch()) return false;
        return true;
    };
    /* one graph replays epg epochs (about 32 steps: the host launches once per replay); with
     * per-epoch metrics every epoch is its own replay followed by a statistics read */
    const bool metrics = hpnn_metrics_active() != 0;
    const int E = (int)o->epochs;
    const int epg = metrics ? 1 : std::max(1, std::min(E, 32 / std::max(1, n_batches)));
    hpnn_preload_code_objects();
    std::map<int, hipGraphExec_t> graphs;
    if (graphs_enabled() && n_batches <= 4096)
        for (int ne : {epg, E % epg}) {
            if (ne <= 0 || graphs.count(ne)) continue;
            hipGraphExec_t x = nullptr;
            if (!capture_epoch(s, [&]() { return epochs(ne); }, &x))
                NN_DBG(stdout, "batched GPU training: epochs not capturable, eager launches\n");
            graphs[ne] = x;
        }
    /* setup (data upload and layout conversions) is finished before the clock starts */
    HIPCHK(hipDeviceSynchronize());
    auto t0 = std::chrono::steady_clock::now();
    double ep_loss = 0.0;
    unsigned int ep_hits = 0;
    BOOL ok = TRUE;
    /* hand-off health after every replay (<= ~32 steps): a 12-byte readback enqueued behind the
     * replay and judged one replay later (the host has already queued the next replay, so the
     * GPU never waits for the check), plus a final check after the last replay */
    unsigned int *hw = nullptr;
    hipEvent_t hev[2] = {nullptr, nullptr};
    if (hipHostMalloc((void **)&hw, 8 * sizeof(unsigned int), hipHostMallocDefault) != hipSuccess ||
        hipEventCreateWithFlags(&hev[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&hev[1], hipEventDisableTiming) != hipSuccess)
        ok = FALSE;
    int pend = -1, slot = 0;
    auto judge = [&](int sl) -> bool { return hipEventSynchronize(hev[sl]) == hipSuccess && net.health_ok(hw + 4 * sl); };
    for (int e = 0; e < E && ok;) {
        const int ne = std::min(epg, E - e);
        auto g = graphs.find(ne);
        ok = (g != graphs.end() && g->second) ? hipGraphLaunch(g->second, s) == hipSuccess : epochs(ne);
        e += ne;
        if (ok) {
            unsigned int *d = hw + 4 * slot;
            d[0] = d[1] = d[2] = 0;
            ok = net.health_enqueue(d) && hipEventRecord(hev[slot], s) == hipSuccess;
        }
        if (ok && pend >= 0) ok = judge(pend);
        pend = ok ? slot : -1;
        slot ^= 1;
        if (ok && (metrics || e == E)) {
            ok = judge(pend); /* statistics read = a synchronisation anyway: judge this replay now */
            pend = -1;
            if (ok) ok = net.read_stats(&ep_loss, &ep_hits);
        }
        if (ok && metrics)
            hpnn_metrics_epoch("gpu", o->epoch0 + e, ep_loss / (double)n, ep_hits, n,
                               std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(),
                               (UINT64)n * e);
    }
    if (ok && pend >= 0) ok = judge(pend);
    auto t1 = std::chrono::steady_clock::now();
    for (hipEvent_t ev : hev)
        if (ev) hipEventDestroy(ev);
    if (hw) hipHostFree(hw);
    for (auto &g : graphs)
        if (g.second) hipGraphExecDestroy(g.second);
    if (ok) ok = net.download(k);
    if (ok && st) {
        st->seconds = std::chrono::duration<double>(t1 - t0).count();
        st->samples = (UINT64)n * o->epochs;
        st->epoch_loss = ep_loss / (double)n;
        st->correct = ep_hits;
        st->last_loss = st->epoch_loss;
    }
    xs.release();
    hpnn_dev_free(Td);
    /* device FP64 copy of the online engine (if any) is now stale */
    if (k->gpu) ((GpuModel *)k->gpu)->host_newer = true;
    return ok;
}

}  // namespace

namespace {

template <class Net>
BOOL train_dp(kernel_ann *k, const DOUBLE *X, const DOUBLE *T, UINT n, const hpnn_batched_opts *o,
              hpnn_batched_stats *st, int G, bool loopback) {
    typedef typename Net::target_t TT;
    typedef typename Net::grad_t GT;
    if (k->n_hiddens + 1 > 16 || G < 1) return FALSE;
    if (!loopback && !hpnn_comm_available()) return FALSE;
    hpnn_gpu_sync_host(k);
    const int B = (int)(o->batch ? o->batch : 256);
    const int Bg = (B + G - 1) / G;
    const bool mom = o->train == NN_TRAIN_BPM;
    const int n_out = (int)k->n_outputs;
    std::vector<int> dev(G);
    std::vector<hipStream_t> str(G);
    std::vector<std::unique_ptr<Net>> nets(G);
    GT *lb_flat = nullptr; /* loopback: [G][count] in one allocation */
    std::vector<XSet> Xd(G);
    std::vector<TT *> Td(G, nullptr);
    std::vector<hpnn_comm *> comms(G, nullptr);
    BOOL ok = TRUE;
    const int n_batches = (int)((n + B - 1) / B);
    auto cleanup = [&]() {
        for (int g = 0; g < G; g++) {
            hipSetDevice(dev[g]);
            if (!loopback || g == 0) {
                Xd[g].release();
                hpnn_dev_free(Td[g]);
            }
            nets[g].reset();
            if (comms[g]) hpnn_comm_destroy(comms[g]);
        }
        if (lb_flat) hpnn_dev_free(lb_flat);
        hipSetDevice(hpnn_rt_device(0));
    };
    for (int g = 0; g < G; g++) {
        dev[g] = loopback ? hpnn_rt_device(0) : hpnn_rt_device((UINT)g);
        str[g] = loopback ? hpnn_rt_stream(0, 0) : hpnn_rt_stream((UINT)g, 0);
        if (!str[g]) return FALSE;
    }
    /* replicas + data (rows padded so every shard of the last minibatch reads Bp rows) */
    const int rows_p = n_batches * B + Bg + 128;
    for (int g = 0; g < G && ok; g++) {
        if (hipSetDevice(dev[g]) != hipSuccess) return FALSE;
        nets[g].reset(new Net());
        /* fragment-major inputs need every shard to start at a multiple of 32 rows */
        ok = nets[g]->init(k, Bg, o->type, mom, str[g], B % 32 == 0 && Bg % 32 == 0);
        if (ok && mom && o->resume) ok = nets[g]->upload_momentum(k);
        if (!ok) break;
        if (loopback) {
            if (g == 0) {
                size_t tot = 0;
                if (!nets[0]->alloc_flat(nullptr)) ok = FALSE; /* sizes only; re-pointed below */
                if (ok) tot = nets[0]->flat_count();
                if (ok && hpnn_dev_malloc(&lb_flat, tot * sizeof(GT) * G) != hipSuccess) ok = FALSE;
            }
            if (ok) {
                const size_t tot = nets[0]->flat_count();
                if (g == 0 && nets[0]->own_flat) {
                    hpnn_dev_free(nets[0]->gflat);
                    nets[0]->own_flat = false;
                }
                ok = nets[g]->alloc_flat(lb_flat + tot * g);
            }
        } else {
            ok = nets[g]->alloc_flat();
        }
        if (!ok) break;
        if (!loopback || g == 0) {
            ok = nets[g]->upload_x(X, (int)n, (int)k->n_inputs, rows_p, &Xd[g]);
            if (ok) ok = attach_labels(&Xd[g], T, n, n_out, rows_p, o->type, str[g]);
            if (ok) {
                std::vector<TT> tf((size_t)rows_p * n_out, (TT)0);
                for (size_t i = 0; i < (size_t)n * n_out; i++) tf[i] = (TT)T[i];
                ok = hpnn_dev_malloc(&Td[g], tf.size() * sizeof(TT)) == hipSuccess &&
                     hipMemcpy(Td[g], tf.data(), tf.size() * sizeof(TT), hipMemcpyHostToDevice) == hipSuccess;
            }
        } else {
            Xd[g] = Xd[0];
            Td[g] = Td[0];
        }
    }
    if (ok && !loopback) {
        if (hpnn_comm_init_all(comms.data(), G, dev.data()) != 0) ok = FALSE;
    }
    if (!ok) {
        cleanup();
        return FALSE;
    }
    const size_t count = nets[0]->flat_count();
    NN_OUT(stdout, "data-parallel batched training: %d replicas (%s, %s), %d samples per replica per step\n", G,
           loopback ? "loopback on one GPU" : "RCCL all-reduce", Net::name(), Bg);
    for (int g = 0; g < G; g++) {
        hipSetDevice(dev[g]);
        hpnn_preload_code_objects();
    }
    hipSetDevice(dev[0]);
    auto t0 = std::chrono::steady_clock::now();
    double ep_loss = 0.0;
    unsigned int ep_hits = 0;
    /* RCCL replicas: one HIP graph per replica epoch (HPNN_GRAPH=0: eager) */
    const bool dp_graphs = !loopback && graphs_enabled() && n_batches <= 4096;
    std::vector<hipGraphExec_t> gexec(G, nullptr);
    std::vector<int> gtried(G, 0);
    for (UINT e = 0; e < o->epochs && ok; e++) {
        for (int g = 0; g < G; g++) {
            hipSetDevice(dev[g]);
            hipMemsetAsync(nets[g]->acc, 0, Net::ACC_BYTES, str[g]);
        }
        if (loopback) {
            for (int b = 0; b < n_batches && ok; b++) {
                const int end = (b * B + B < (int)n) ? b * B + B : (int)n;
                int total = 0;
                for (int g = 0; g < G && ok; g++) {
                    const int start = b * B + g * Bg;
                    int nv = end - start;
                    nv = nv < 0 ? 0 : (nv > Bg ? Bg : nv);
                    total += nv;
                    const TT *tb = Td[g] + (size_t)start * n_out;
                    ok = nets[g]->grads(Xd[g], start, tb, n_out, nv);
                }
                if (!ok) break;
                /* virtual replicas share one stream: sum the G buffers into replica 0's */
                ok = Net::reduce_sum(lb_flat, G, count, str[0]) == 0;
                const double scale = 1.0 / (double)(total > 0 ? total : 1);
                for (int g = 0; g < G && ok; g++) ok = nets[g]->update_flat(lb_flat, o->lr, o->alpha, scale, mom);
            }
        } else {
            /* one host thread per GPU for the whole epoch (no serial hipSetDevice + launch
             * loop over the replicas); each layer's bucket goes into an async all-reduce on
             * the communicator's side stream as soon as it is final (last layer first), so
             * it overlaps the backward of the layers below; the update waits on a join */
            std::vector<int> tok(G, 1);
            std::vector<std::thread> th;
            for (int g = 0; g < G; g++)
                th.emplace_back([&, g]() {
                    if (hipSetDevice(dev[g]) != hipSuccess) {
                        tok[g] = 0;
                        return;
                    }
                    Net &net = *nets[g];
                    /* the replica's epoch (HIP graph: captured on the first epoch, the RCCL
                     * collectives and the side-stream fork / join included; replayed after) */
                    auto epoch_body = [&]() -> bool {
                    for (int b = 0; b < n_batches; b++) {
                        const int end = (b * B + B < (int)n) ? b * B + B : (int)n;
                        const int start = b * B + g * Bg;
                        int nv = end - start;
                        nv = nv < 0 ? 0 : (nv > Bg ? Bg : nv);
                        const int total = end - b * B;
                        const TT *tb = Td[g] + (size_t)start * n_out;
                        const std::vector<std::pair<int, int>> seq = net.buckets();
                        size_t issued = 0;
                        auto ready = [&](int lo, int hi) {
                            issued++;
                            return hpnn_comm_all_reduce_async(comms[g], net.gflat + net.goff[lo],
                                                              (long)(net.goff[hi + 1] - net.goff[lo]), Net::comm_dt,
                                                              str[g]) == 0;
                        };
                        /* after a local failure every remaining bucket is still all-reduced (same
                         * sizes, same order on every replica), so no peer is left waiting */
                        int okb = tok[g] && net.grads(Xd[g], start, tb, n_out, nv, ready) ? 1 : 0;
                        for (size_t i = issued; i < seq.size(); i++) ready(seq[i].first, seq[i].second);
                        okb = (hpnn_comm_join(comms[g], str[g]) == 0) && okb;
                        const double scale = 1.0 / (double)(total > 0 ? total : 1);
                        okb = okb && net.update_flat(net.gflat, o->lr, o->alpha, scale, mom);
                        if (!okb && tok[g]) {
                            NN_ERROR(stderr, "data-parallel step failed on replica %d\n", g);
                            tok[g] = 0;
                        }
                    }
                    return tok[g] != 0;
                    };
                    if (dp_graphs && !gtried[g]) {
                        gtried[g] = 1;
                        if (!capture_epoch(str[g], epoch_body, &gexec[g]))
                            NN_DBG(stdout, "data-parallel replica %d: epoch not capturable, eager launches\n", g);
                    }
                    if (gexec[g]) {
                        if (hipGraphLaunch(gexec[g], str[g]) != hipSuccess) tok[g] = 0;
                    } else {
                        epoch_body();
                    }
                    if (hipStreamSynchronize(str[g]) != hipSuccess) tok[g] = 0;
                });
            for (auto &t : th) t.join();
            for (int g = 0; g < G; g++) ok = ok && tok[g];
        }
        if (!ok) break;
        ep_loss = 0.0;
        ep_hits = 0;
        for (int g = 0; g < G && ok; g++) {
            hipSetDevice(dev[g]);
            double l = 0.0;
            unsigned int h = 0;
            ok = nets[g]->read_stats(&l, &h) && nets[g]->healthy();
            ep_loss += l;
            ep_hits += h;
        }
        if (!loopback && ok) {
            /* surface asynchronous communicator failures (a peer died, link error) */
            for (int g = 0; g < G; g++)
                if (hpnn_comm_check(comms[g]) != 0) ok = FALSE;
        }
        if (ok && hpnn_metrics_active())
            hpnn_metrics_epoch(loopback ? "gpu-dp-loopback" : "gpu-dp", o->epoch0 + e + 1, ep_loss / (double)n,
                               ep_hits, n, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(),
                               (UINT64)n * (e + 1));
    }
    auto t1 = std::chrono::steady_clock::now();
    for (int g = 0; g < G; g++)
        if (gexec[g]) {
            hipSetDevice(dev[g]);
            hipGraphExecDestroy(gexec[g]);
        }
    if (ok) {
        hipSetDevice(dev[0]);
        ok = nets[0]->download(k);
    }
    if (ok && st) {
        st->seconds = std::chrono::duration<double>(t1 - t0).count();
        st->samples = (UINT64)n * o->epochs;
        st->epoch_loss = ep_loss / (double)n;
        st->correct = ep_hits;
        st->last_loss = st->epoch_loss;
    }
    cleanup();
    if (ok && k->gpu) ((GpuModel *)k->gpu)->host_newer = true;
    return ok;
}

/* Data parallelism with ONE process per GPU (any launcher exporting RANK / WORLD_SIZE /
 * LOCAL_RANK; the reference ran `mpirun -np N train_nn` and replicated the same sample on
 * every rank).  Rank r trains rows [b*B + r*ceil(B/W), ...) of every global
 * minibatch b; the FP32 gradients are summed with the one-shot xGMI all-reduce (all
 * ranks on one node, gradients <= 4 MiB) or RCCL, the bootstrap exchange (IPC handles /
 * unique id / epoch statistics) goes through include/libhpnn/bootstrap.h; every rank
 * applies the same update, so the weights stay identical (rank 0 writes the files). */
template <class Net>
BOOL train_dp_mp(kernel_ann *k, const DOUBLE *X, const DOUBLE *T, UINT n, const hpnn_batched_opts *o,
                 hpnn_batched_stats *st) {
    typedef typename Net::target_t TT;
    const int W = hpnn_boot_world(), R = hpnn_boot_rank();
    if (k->n_hiddens + 1 > 16 || W < 1 || W > 64) return FALSE;
    hpnn_gpu_sync_host(k);
    const int dev = hpnn_rt_device(0);
    HIPCHK(hipSetDevice(dev));
    hipStream_t s = hpnn_rt_stream(0, 0);
    const int B = (int)(o->batch ? o->batch : 256);
    const int Bg = (B + W - 1) / W;
    const bool mom = o->train == NN_TRAIN_BPM;
    const int n_out = (int)k->n_outputs;
    /* HPNN_GRAD_COMM=bf16rs: BF16 reduce-scatter + sharded step + BF16 all-gather (RCCL,
     * per-layer plan); fp32: the FP32 all-reduce; auto (default): bf16rs for the BF16 engine
     * when the net takes the per-layer plan and its FP32 gradients exceed 4 MB (bandwidth-
     * bound exchange: half the bytes, each rank steps 1 / world of the rows), else fp32.
     * Every rank reads the same environment and net, so all decide alike. */
    const char *gce = getenv("HPNN_GRAD_COMM");
    bool bf16rs = gce && !strcmp(gce, "bf16rs");
    if (!gce || !strcmp(gce, "auto")) {
        double gbytes = 0.0;
        const int nl = (int)k->n_hiddens + 1;
        std::vector<int> sizes(nl + 1);
        sizes[0] = (int)k->n_inputs;
        for (int l = 0; l < nl; l++) {
            sizes[l + 1] = (int)layer_of(k, l)->n_neurons;
            gbytes += 4.0 * sizes[l] * sizes[l + 1];
        }
        hpnn::BPlan probe; /* host-only configuration: which step structure the net gets */
        const int ty = o->type == NN_TYPE_ANN ? 0 : (o->type == NN_TYPE_LNN ? 1 : 2);
        const bool per_layer =
            probe.configure(sizes.data(), nl, ty, Bg, mom, -1, nullptr, 512, false) == 0 && probe.mode == 0;
        bf16rs = W > 1 && !strcmp(Net::name(), "bf16") && per_layer && gbytes > (double)(4 << 20);
    }
    Net net;
    if (!net.init(k, Bg, o->type, mom, s, B % 32 == 0 && Bg % 32 == 0, bf16rs ? 0 : -1) || !net.alloc_flat())
        return FALSE;
    if (mom && o->resume && !net.upload_momentum(k)) return FALSE;
    const size_t count = net.flat_count();
    /* gradient exchange: one-shot xGMI all-reduce when every rank is on this node and the
     * gradients are small, else RCCL; every rank takes the same decision */
    hpnn_xar *xar = nullptr, *xark = nullptr;
    hpnn_comm *comm = nullptr;
    const char *xe = getenv("HPNN_XAR");
    const char *lws = getenv("LOCAL_WORLD_SIZE");
    /* the xGMI all-reduce sums FP32; FP64 gradients go through RCCL */
    bool use_xar = Net::comm_dt == HPNN_DT_F32 && !(xe && xe[0] == '0') && lws && atoi(lws) == W &&
                   W <= HPNN_XAR_MAX_RANKS && count * 4 <= ((size_t)4 << 20) && !bf16rs;
    /* collective: create, exchange the IPC handles, open, self-test on the real links; every
     * rank agrees, else all get nullptr (-1: bootstrap failure) */
    auto open_xar = [&](size_t bytes, hpnn_xar **out) -> int {
        *out = nullptr;
        hpnn_xar *x = hpnn_xar_create(R, W, bytes);
        std::vector<char> h(HPNN_XAR_HANDLE_BYTES, 0), all((size_t)W * HPNN_XAR_HANDLE_BYTES);
        int ok = x && hpnn_xar_handles(x, h.data()) == 0;
        if (hpnn_boot_allgather(h.data(), h.size(), all.data()) != 0) return -1;
        if (ok) ok = hpnn_xar_open(x, all.data()) == 0;
        std::vector<int> oks(W);
        if (hpnn_boot_allgather(&ok, sizeof ok, oks.data()) != 0) return -1;
        bool all_ok = true;
        for (int v : oks) all_ok = all_ok && v;
        if (all_ok) { /* known sums over the real links before any gradient goes through */
            const int rc = hpnn_xar_self_test(x, s);
            ok = rc == 0;
            if (!ok) NN_WARN(stderr, "xGMI all-reduce self-test failed (%d) on rank %d\n", rc, R);
            if (hpnn_boot_allgather(&ok, sizeof ok, oks.data()) != 0) return -1;
            for (int v : oks) all_ok = all_ok && v;
        }
        if (!all_ok) {
            if (x) hpnn_xar_destroy(x);
            return 0;
        }
        *out = x;
        return 0;
    };
    if (use_xar) {
        if (open_xar(count * 4, &xar)) return FALSE;
        use_xar = xar != nullptr;
        /* fused modes: a second communicator whose protocol runs inside the G0 launch
         * (HPNN_XAR_G0=0: the all-reduce launch instead) */
        const char *xg = getenv("HPNN_XAR_G0");
        if (use_xar && !(xg && xg[0] == '0') && open_xar(count * 4, &xark)) return FALSE;
    }
    /* collective: the RCCL communicator (rank 0's unique id through the bootstrap) */
    auto open_rccl = [&]() -> bool {
        unsigned char id[HPNN_COMM_ID_BYTES] = {0};
        std::vector<unsigned char> all((size_t)W * HPNN_COMM_ID_BYTES);
        if (R == 0 && hpnn_comm_unique_id(id) != 0) return false;
        if (hpnn_boot_allgather(id, sizeof id, all.data()) != 0) return false;
        comm = hpnn_comm_init_rank(all.data(), W, R, dev); /* rank 0's id */
        if (!comm) return false;
        /* BF16 batched engine: the library's overlapped data-parallel step (dp_exchange.h);
         * FP32 / FP64 engines: the bucket loop below */
        if (!net.attach_dpx(comm, bf16rs ? hpnn::DpExchange::BF16RS : hpnn::DpExchange::FP32) && bf16rs)
            NN_WARN(stderr, "bf16rs exchange unavailable for this net: FP32 all-reduce\n");
        return true;
    };
    if (!use_xar && !open_rccl()) return FALSE;
    NN_OUT(stdout, "data-parallel batched training: %d processes (%s, %s), %d samples per rank per step\n", W,
           use_xar ? "xGMI all-reduce" : "RCCL all-reduce", Net::name(), Bg);
    /* the gradient exchange chosen (HPNN_GRAD_COMM; auto picks bf16rs for large per-layer nets) */
    if (R == 0 && W > 1)
        NN_OUT(stdout, "data-parallel gradient exchange: %s\n",
               bf16rs ? "bf16rs (BF16 reduce-scatter, sharded FP32 step, BF16 all-gather)" : "fp32 (all-reduce)");
    const int n_batches = (int)((n + B - 1) / B);
    const int rows_p = n_batches * B + Bg + 128;
    XSet Xd;
    TT *Td = nullptr;
    BOOL ok = net.upload_x(X, (int)n, (int)k->n_inputs, rows_p, &Xd);
    if (ok) ok = attach_labels(&Xd, T, n, n_out, rows_p, o->type, s);
    if (ok) {
        std::vector<TT> tf((size_t)rows_p * n_out, (TT)0);
        for (size_t i = 0; i < (size_t)n * n_out; i++) tf[i] = (TT)T[i];
        ok = hpnn_dev_malloc(&Td, tf.size() * sizeof(TT)) == hipSuccess &&
             hipMemcpy(Td, tf.data(), tf.size() * sizeof(TT), hipMemcpyHostToDevice) == hipSuccess;
    }
    hpnn_preload_code_objects();
    /* per-replay health: plan hand-off words [0..2], exchange error words [3..4], per slot */
    unsigned int *hw = nullptr;
    hipEvent_t hev[2] = {nullptr, nullptr};
    if (hipHostMalloc((void **)&hw, 16 * sizeof(unsigned int), hipHostMallocDefault) != hipSuccess ||
        hipEventCreateWithFlags(&hev[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&hev[1], hipEventDisableTiming) != hipSuccess)
        ok = FALSE;
    int pend = -1; /* slot whose readback is in flight */
    auto enqueue_check = [&](int slot) -> bool {
        unsigned int *d = hw + 8 * slot;
        for (int i = 0; i < 8; i++) d[i] = 0;
        bool r = net.health_enqueue(d);
        if (r && use_xar) r = hpnn_xar_status_enqueue(xar, d + 3, s) == 0;
        if (r && xark) r = hpnn_xar_status_enqueue(xark, d + 4, s) == 0;
        return r && hipEventRecord(hev[slot], s) == hipSuccess;
    };
    auto finish_check = [&](int slot) -> bool {
        if (hipEventSynchronize(hev[slot]) != hipSuccess) return false;
        const unsigned int *d = hw + 8 * slot;
        if (!net.health_ok(d)) return false;
        return use_xar ? d[3] == 0 && d[4] == 0 : hpnn_comm_check(comm) == 0;
    };
    /* preflight: the plan and the exchange start clean (and the first reads of their words, a
     * few ms while the runtime maps them, stay out of the training time) */
    if (ok) ok = enqueue_check(0) && finish_check(0);
    {
        /* ... and every other readback of the agreement points once (statistics, digest):
         * their first calls set up host staging and copy paths (ms) */
        double l0 = 0.0;
        unsigned int h0 = 0;
        unsigned long long d0 = 0;
        if (ok) ok = net.read_stats(&l0, &h0) && net.digest(&d0);
    }
    /* setup (data upload and layout conversions) is finished before the clock starts */
    if (hipDeviceSynchronize() != hipSuccess) ok = FALSE;
    auto t0 = std::chrono::steady_clock::now();
    double ep_loss = 0.0;
    unsigned int ep_hits = 0;
    /* one epoch's steps: the same launches on every rank, every epoch (the minibatch order is
     * fixed), so from the second epoch on they replay as ONE HIP graph per epoch -- the
     * launches bench.py times (the first epoch runs eagerly: it settles the exchange form) */
    /* reset: zero the statistics first (only the last epoch of a replay group is ever read) */
    auto epoch_steps = [&](UINT e, bool reset = true) -> bool {
        if (reset && hipMemsetAsync(net.acc, 0, Net::ACC_BYTES, s) != hipSuccess) return false;
        for (int b = 0; b < n_batches; b++) {
            const int end = (b * B + B < (int)n) ? b * B + B : (int)n;
            const int start = b * B + R * Bg;
            int nv = end - start;
            nv = nv < 0 ? 0 : (nv > Bg ? Bg : nv);
            const TT *tb = Td + (size_t)start * n_out;
            const int total = end - b * B;
            if (net.has_dpx()) {
                if (!net.dp_step(Xd, start, tb, n_out, nv, total, o->lr, o->alpha)) return false;
                continue;
            }
            if (xark) {
                /* the exchange and every step inside the first-layer gradient launch */
                const int r = net.xchg_step(Xd, start, tb, n_out, nv, o->lr, o->alpha,
                                            1.0 / (double)(total > 0 ? total : 1), xark);
                if (r == 0) {
                    if (e == 0 && b == 0 && R == 0)
                        NN_OUT(stdout, "data-parallel step: exchange inside the first-layer gradient launch\n");
                    continue;
                }
                if (r != -1) {
                    NN_ERROR(stderr, "data-parallel fused step failed: %d\n", r);
                    return false;
                }
                /* not covered (same on every rank): the all-reduce launch from here on */
                hpnn_xar_destroy(xark);
                xark = nullptr;
            }
            bool okb;
            if (use_xar) {
                /* small gradients: ONE latency-bound xGMI all-reduce of the whole buffer */
                okb = net.grads(Xd, start, tb, n_out, nv) &&
                      hpnn_xar_all_reduce_f32(xar, (float *)net.gflat, (float *)net.gflat, (long)count, s) == 0;
            } else {
                /* RCCL: one bucket per layer on the side stream as soon as it is final
                 * (overlapping the backward of the layers below); the update joins them */
                const std::vector<std::pair<int, int>> seq = net.buckets();
                size_t issued = 0;
                auto ready = [&](int lo, int hi) {
                    issued++;
                    return hpnn_comm_all_reduce_async(comm, net.gflat + net.goff[lo],
                                                      (long)(net.goff[hi + 1] - net.goff[lo]), Net::comm_dt, s) == 0;
                };
                okb = net.grads(Xd, start, tb, n_out, nv, ready);
                for (size_t i = issued; i < seq.size(); i++) ready(seq[i].first, seq[i].second);
                okb = (hpnn_comm_join(comm, s) == 0) && okb;
            }
            if (!okb || !net.update_flat(net.gflat, o->lr, o->alpha, 1.0 / (double)(total > 0 ? total : 1), mom))
                return false;
        }
        return true;
    };
    /* Epoch 0 runs eagerly; then one HIP graph replays epg epochs (about 32 steps, as
     * train_single).  After every replay a rank checks its own health (one small readback);
     * the ranks agree (one host all-gather) after the first epoch, the last, every epoch under
     * metrics and every 16th replay otherwise.  Between agreements a rank that saw a failure
     * keeps launching -- the exchange needs every rank in step -- and reports it at the next
     * one.  Graph capture is setup, not training: its time is left out of the training time,
     * as train_single captures before its clock starts. */
    const bool metrics = hpnn_metrics_active() != 0;
    const UINT E = o->epochs;
    const UINT epg = metrics ? 1u : std::max(1u, std::min(E > 1 ? E - 1 : 1u, 32u / (UINT)std::max(1, n_batches)));
    hipGraphExec_t gx = nullptr;
    double setup_s = 0.0;
    bool local_ok = true;
    bool recheck = false; /* digests compared again at the next agreement point (after a fallback) */
    UINT replays = 0;
    for (UINT e = 0; e < E && ok;) {
        if (e == 1 && graphs_enabled() && n_batches <= 4096 && E - 1 >= epg) {
            /* every rank captures; all replay only if all captured (a failed capture ran
             * nothing, so eager epochs stay in step) */
            const auto c0 = std::chrono::steady_clock::now();
            int cap = capture_epoch(s, [&]() {
                for (UINT i = 0; i < epg; i++)
                    if (!epoch_steps(e + i, i + 1 == epg)) return false;
                return true;
            }, &gx) ? 1 : 0;
            std::vector<int> caps(W);
            if (hpnn_boot_allgather(&cap, sizeof cap, caps.data()) != 0) ok = FALSE;
            for (int v : caps) cap = cap && v;
            if (!cap && gx) {
                hipGraphExecDestroy(gx);
                gx = nullptr;
            }
            if (ok && R == 0)
                NN_OUT(stdout, "data-parallel epochs: %s\n", gx ? "HIP graph replays" : "eager launches (capture failed)");
            setup_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - c0).count();
            if (!ok) break;
        }
        const UINT ne = e == 0 ? 1u : std::min(epg, E - e);
        bool lok;
        if (gx && e > 0 && ne == epg) {
            lok = hipGraphLaunch(gx, s) == hipSuccess;
        } else {
            lok = true;
            for (UINT i = 0; i < ne && lok; i++) lok = epoch_steps(e + i, i + 1 == ne);
        }
        e += ne;
        if (e > 1) replays++;
        /* this replay's health words are read back behind it; the previous replay's are judged
         * now (the host waits for that replay only, with this one queued behind it) */
        const int slot = (int)(replays & 1);
        if (lok) lok = enqueue_check(slot);
        if (pend >= 0) local_ok = finish_check(pend) && local_ok;
        pend = lok ? slot : -1;
        local_ok = local_ok && lok;
        const bool first = e == 1, last = e == E;
        if (!(first || last || metrics || recheck || replays % 16 == 0)) continue;
        /* agreement point */
        if (pend >= 0) local_ok = finish_check(pend) && local_ok;
        pend = -1;
        double l = 0.0;
        unsigned int h = 0;
        if (local_ok && !net.read_stats(&l, &h)) local_ok = false;
        /* replicas must hold bitwise-identical weights: a wrong-but-timely exchange (a sum that
         * arrived in time but is not every rank's) shows here, after the first epoch and the last */
        unsigned long long dig = 0;
        const bool check_dig = first || last || recheck;
        if (local_ok && check_dig && !net.digest(&dig)) local_ok = false;
        if (local_ok && check_dig && R == W - 1 && hpnn_fault_hit("digest")) dig ^= 1; /* test hook */
        if (local_ok && check_dig && first && R == W - 1 && use_xar && hpnn_fault_hit("xdigest"))
            dig ^= 1; /* test hook: the first xGMI epoch looks wrong on one rank -> fallback */
        struct {
            double loss;
            unsigned long long digest;
            unsigned int hits, ok;
        } mine = {l, dig, h, (unsigned)local_ok}, *every = new decltype(mine)[W];
        if (hpnn_boot_allgather(&mine, sizeof mine, every) != 0) ok = FALSE;
        ep_loss = 0.0;
        ep_hits = 0;
        bool same = true;
        for (int r = 0; r < W && ok; r++) {
            ep_loss += every[r].loss;
            ep_hits += every[r].hits;
            ok = ok && every[r].ok;
            same = same && every[r].digest == every[0].digest;
        }
        delete[] every;
        if (first && R == 0)
            NN_DBG(stdout, "data-parallel: epoch 1 (eager, with the weight digest) %.3f ms\n",
                   1e3 * std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
        if (ok && check_dig && !same && first && use_xar) {
            /* a wrong-but-timely xGMI sum: degrade instead of stopping -- every rank leaves the
             * xGMI exchange for RCCL, rank 0's weights and momentum are re-broadcast, and the
             * digests are compared again after the next epoch (a mismatch there stops the run).
             * Reference: the P2P -> CMM -> EXP fallback chain, libhpnn.c:245-302 */
            if (R == 0)
                NN_WARN(stderr, "data-parallel training: the replicas' weights differ after epoch 1 over the "
                                "xGMI exchange; falling back to RCCL from rank 0's weights\n");
            std::vector<char> mine_st, all_st;
            ok = net.get_state(mine_st);
            if (ok) {
                all_st.resize(mine_st.size() * (size_t)W);
                ok = hpnn_boot_allgather(mine_st.data(), mine_st.size(), all_st.data()) == 0 &&
                     net.set_state(all_st.data()); /* rank 0's block */
            }
            if (xark) hpnn_xar_destroy(xark);
            if (xar) hpnn_xar_destroy(xar);
            xark = xar = nullptr;
            use_xar = false;
            if (ok && !open_rccl()) ok = FALSE;
            recheck = true;
            same = true;
        } else if (ok && check_dig && recheck) {
            recheck = false;
        }
        if (ok && check_dig && !same) {
            if (R == 0)
                NN_ERROR(stderr, "data-parallel training: the replicas' weights differ after epoch %u "
                                 "(exchange error); stopping\n", e);
            ok = FALSE;
        }
        if (ok && metrics)
            hpnn_metrics_epoch("gpu-dp-mp", o->epoch0 + e, ep_loss / (double)n, ep_hits, n,
                               std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() - setup_s,
                               (UINT64)n * e);
    }
    auto t1 = std::chrono::steady_clock::now();
    if (gx) hipGraphExecDestroy(gx);
    hipStreamSynchronize(s);
    for (hipEvent_t ev : hev)
        if (ev) hipEventDestroy(ev);
    if (hw) hipHostFree(hw);
    if (ok) ok = net.gather_masters(); /* bf16rs: every rank's rows of the FP32 masters */
    if (ok) ok = net.download(k);
    if (ok && st) {
        st->seconds = std::chrono::duration<double>(t1 - t0).count() - setup_s;
        st->samples = (UINT64)n * o->epochs;
        st->epoch_loss = ep_loss / (double)n;
        st->correct = ep_hits;
        st->last_loss = st->epoch_loss;
    }
    hipStreamSynchronize(s);
    net.detach_dpx(); /* before the communicator goes */
    hpnn_boot_finish(); /* every rank is past its last all-reduce before any buffer goes */
    Xd.release();
    if (Td) hpnn_dev_free(Td);
    if (xar) hpnn_xar_destroy(xar);
    if (xark) hpnn_xar_destroy(xark);
    if (comm) hpnn_comm_destroy(comm);
    if (ok && k->gpu) ((GpuModel *)k->gpu)->host_newer = true;
    return ok;
}

}  // namespace

namespace {

BOOL infer_bf16(kernel_ann *k, nn_type type, const DOUBLE *X, UINT n, DOUBLE *Y, hipStream_t s) {
    const int B = 4096;
    Batched net;
    if (!net.init(k, B, type, false, s, false, 0)) return FALSE; /* forward only: per-layer plan */
    const int n_batches = (int)((n + B - 1) / B);
    const int rows_p = (n_batches - 1) * B + net.Bp;
    const int no = net.p.Np[net.L - 1];
    XSet xs;
    float *O = nullptr;
    if (!net.upload_x(X, (int)n, (int)k->n_inputs, rows_p, &xs)) return FALSE;
    HIPCHK(hpnn_dev_malloc(&O, (size_t)net.Bp * no * 4));
    std::vector<float> h((size_t)net.Bp * no);
    BOOL ok = TRUE;
    for (int b = 0; b < n_batches && ok; b++) {
        const int nv = (b == n_batches - 1) ? (int)n - b * B : B;
        ok = net.p.predict(net.at(xs, (long)b * B).x, nv, O, no, s) == 0;
        ok = ok && hipMemcpyAsync(h.data(), O, h.size() * 4, hipMemcpyDeviceToHost, s) == hipSuccess &&
             hipStreamSynchronize(s) == hipSuccess;
        for (int r = 0; ok && r < nv; r++)
            for (UINT c = 0; c < k->n_outputs; c++) Y[((size_t)b * B + r) * k->n_outputs + c] = h[(size_t)r * no + c];
    }
    xs.release();
    hpnn_dev_free(O);
    return ok;
}

/* FP64 / FP32 inference: the forward GEMMs and the output activation in the model's
 * precision, one device-to-host copy of the outputs per block of samples */
template <typename T>
BOOL infer_fp(kernel_ann *k, nn_type type, const DOUBLE *X, UINT n, DOUBLE *Y, hipStream_t s) {
    const int B = (int)(n < 16384 ? n : 16384);
    BatchedFP<T> net;
    if (!net.init(k, B, type, false, s)) return FALSE;
    const int n_batches = (int)((n + B - 1) / B);
    const int rows_p = n_batches * B;
    const int no = (int)k->n_outputs;
    XSet xs;
    T *O = nullptr;
    if (!net.upload_x(X, (int)n, (int)k->n_inputs, rows_p, &xs)) return FALSE;
    HIPCHK(hpnn_dev_malloc(&O, (size_t)B * no * sizeof(T)));
    std::vector<T> h((size_t)B * no);
    BOOL ok = TRUE;
    for (int b = 0; b < n_batches && ok; b++) {
        const int nv = (b == n_batches - 1) ? (int)n - b * B : B;
        ok = net.forward(BatchedFP<T>::at(xs, (long)b * B), B);
        if (ok)
            ok = hpnn_output_fp(BatchedFP<T>::F64, net.Z, no, nullptr, 0, nullptr, 0, O, no, nullptr, nullptr, nullptr,
                                B, 0, no, net.type, s) == 0;
        ok = ok && hipMemcpyAsync(h.data(), O, (size_t)nv * no * sizeof(T), hipMemcpyDeviceToHost, s) == hipSuccess &&
             hipStreamSynchronize(s) == hipSuccess;
        for (size_t i = 0; ok && i < (size_t)nv * no; i++) Y[(size_t)b * B * no + i] = (DOUBLE)h[i];
    }
    xs.release();
    hpnn_dev_free(O);
    return ok;
}

}  // namespace

/* batched evaluation (run_nn on the GPU): the whole test set through the batched engine
 * of the requested precision instead of one online forward per file.  With n_gpu x
 * n_streams > 1 (run_nn -G N -S M, the reference's forward over n_gpu x n_streams,
 * cuda_ann.cu:426-1276) the samples are split into N M contiguous shards, one host thread
 * each on its own (device, stream) (forward only: no communication; outputs land in
 * place).  HPNN_INFER_SHARDS = V runs V shards on device 0, each on its own new stream
 * (tests on one GPU). */
extern "C" BOOL hpnn_gpu_infer_batched(kernel_ann *k, nn_type type, nn_dtype dtype, const DOUBLE *X, UINT n,
                                       DOUBLE *Y) {
    if (!k || n == 0) return FALSE;
    if (dtype != NN_DTYPE_BF16 && dtype != NN_DTYPE_F32 && dtype != NN_DTYPE_F64) {
        NN_ERROR(stderr, "GPU inference: unsupported dtype %d\n", (int)dtype);
        return FALSE;
    }
    hpnn_gpu_sync_host(k);
    const nn_runtime *rt = hpnn_rt_get();
    const int G = rt && rt->cudas.n_gpu > 1 ? (int)rt->cudas.n_gpu : 1;
    const int NS = rt && rt->cudas.cuda_n_streams > 1 ? (int)rt->cudas.cuda_n_streams : 1;
    const char *vs = getenv("HPNN_INFER_SHARDS");
    const int V = vs ? atoi(vs) : 0;
    const bool virt = V >= 2;
    int P = virt ? V : G * NS;
    if ((UINT)P > n) P = (int)n;
    const UINT ni = k->n_inputs, no = k->n_outputs;
    auto shard = [&](int g, hipStream_t s) -> BOOL {
        const UINT lo = (UINT)((UINT64)n * g / P), hi = (UINT)((UINT64)n * (g + 1) / P);
        if (hi == lo) return TRUE;
        const DOUBLE *Xs = X + (size_t)lo * ni;
        DOUBLE *Ys = Y + (size_t)lo * no;
        switch (dtype) {
        case NN_DTYPE_BF16: return infer_bf16(k, type, Xs, hi - lo, Ys, s);
        case NN_DTYPE_F32: return infer_fp<float>(k, type, Xs, hi - lo, Ys, s);
        default: return infer_fp<double>(k, type, Xs, hi - lo, Ys, s);
        }
    };
    if (P <= 1) {
        HIPCHK(hipSetDevice(hpnn_rt_device(0)));
        return shard(0, hpnn_rt_stream(0, 0));
    }
    NN_DBG(stdout, "batched evaluation: %u samples over %d %s\n", n, P,
           virt ? "shards on one GPU" : "(GPU, stream) shards");
    std::vector<int> ok(P, 0);
    std::vector<std::thread> th;
    for (int g = 0; g < P; g++)
        th.emplace_back([&, g]() {
            /* shard g: device g / NS, stream g % NS (consecutive shards on one device) */
            const int dev = hpnn_rt_device(virt ? 0 : (UINT)(g / NS));
            if (hipSetDevice(dev) != hipSuccess) return;
            hipStream_t s = nullptr;
            if (virt) {
                if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return;
            } else {
                s = hpnn_rt_stream((UINT)(g / NS), (UINT)(g % NS));
            }
            ok[g] = shard(g, s) ? 1 : 0;
            if (virt) hipStreamDestroy(s);
        });
    for (auto &t : th) t.join();
    hipSetDevice(hpnn_rt_device(0));
    for (int g = 0; g < P; g++)
        if (!ok[g]) {
            NN_ERROR(stderr, "batched GPU evaluation: shard %d failed\n", g);
            return FALSE;
        }
    return TRUE;
}
