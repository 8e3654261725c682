/*
 * libhpnn exact training state (checkpoint / resume).
 *
 * The reference checkpoints only the weights, as %17.15f text (kernel.opt, ann.c:770-857;
 * train_nn writes kernel.tmp before and kernel.opt after training, tests/train_nn.c:224-243)
 * and resumes by pointing [init] at that file: momentum, progress and the RNG seed are
 * lost and %17.15f does not round-trip a double (Checkpoint / resume).  The
 * state file keeps kernel.opt as the interchange format and adds a binary sidecar that
 * resumes bit-exactly: FP64 weights, FP64 momentum, seed, epochs / samples done, and a
 * checksum that turns a truncated or corrupted file into a load error.
 *
 * Layout (little endian):
 *   char magic[8] = "HPNNSTA1"
 *   u32 type, train, L (weight layers), has_momentum
 *   u32 dims[L + 1]             n_in, h_1 .. h_{L-1}, n_out
 *   u32 seed, epochs_done, reserved[2]
 *   u64 samples_seen
 *   f64 W_l (N_l x M_l row-major), l = 0 .. L-1
 *   f64 dW_l (same shapes)      when has_momentum
 *   u64 FNV-1a checksum of every byte above
 */
#include <libhpnn/ann.h>
#include <string.h>

#include <string>
#include <vector>

#include "dataset.h"
#include "runtime_internal.h"
#include "../gpu/engine.h"

#define KERN(conf) ((kernel_ann *)((conf)->kernel))
#define STATE_MAGIC "HPNNSTA1"

namespace {

layer_ann *layer_at(kernel_ann *k, UINT l) { return l < k->n_hiddens ? &k->hiddens[l] : &k->output; }

struct Writer {
    std::string buf;
    void put(const void *p, size_t n) { buf.append((const char *)p, n); }
    void u32(UINT v) { put(&v, 4); }
};

struct Reader {
    const std::string &buf;
    size_t off = 0;
    bool ok = true;
    explicit Reader(const std::string &b) : buf(b) {}
    void get(void *p, size_t n) {
        if (!ok || off + n > buf.size()) {
            ok = false;
            return;
        }
        memcpy(p, buf.data() + off, n);
        off += n;
    }
    UINT u32() {
        UINT v = 0;
        get(&v, 4);
        return v;
    }
};

}  // namespace

extern "C" BOOL _NN(dump, state)(nn_def *conf, const CHAR *filename) {
    if (!conf || !conf->kernel || !filename) return FALSE;
    if (hpnn_output_rank() != 0) return TRUE; /* rank 0 writes */
    kernel_ann *k = KERN(conf);
    hpnn_gpu_sync_host(k);
    const UINT L = k->n_hiddens + 1;
    Writer w;
    w.put(STATE_MAGIC, 8);
    w.u32((UINT)conf->type);
    w.u32((UINT)conf->train);
    w.u32(L);
    w.u32(k->dw ? 1u : 0u);
    w.u32(k->n_inputs);
    for (UINT l = 0; l < L; l++) w.u32(layer_at(k, l)->n_neurons);
    w.u32(conf->seed);
    w.u32(conf->epochs_done);
    w.u32(0);
    w.u32(0);
    w.put(&conf->samples_seen, 8);
    for (UINT l = 0; l < L; l++) {
        const layer_ann *ly = layer_at(k, l);
        w.put(ly->weights, sizeof(DOUBLE) * ly->n_neurons * ly->n_inputs);
    }
    if (k->dw)
        for (UINT l = 0; l < L; l++) {
            const layer_ann *ly = layer_at(k, l);
            w.put(k->dw[l], sizeof(DOUBLE) * ly->n_neurons * ly->n_inputs);
        }
    const UINT64 h = hpnn_fnv1a(w.buf.data(), w.buf.size(), HPNN_FNV_SEED);
    w.put(&h, 8);
    /* write to a temporary name, then rename: a crash mid-write never leaves a torn state */
    const std::string tmp = std::string(filename) + ".tmp";
    FILE *fp = fopen(tmp.c_str(), "wb");
    if (!fp) {
        NN_ERROR(stderr, "can't write state file %s\n", tmp.c_str());
        return FALSE;
    }
    bool ok = fwrite(w.buf.data(), 1, w.buf.size(), fp) == w.buf.size();
    ok = (fclose(fp) == 0) && ok;
    if (ok) ok = rename(tmp.c_str(), filename) == 0;
    if (!ok) NN_ERROR(stderr, "can't write state file %s\n", filename);
    return ok ? TRUE : FALSE;
}

extern "C" BOOL _NN(load, state)(nn_def *conf, const CHAR *filename) {
    if (!conf || !conf->kernel || !filename) return FALSE;
    kernel_ann *k = KERN(conf);
    std::string buf;
    {
        FILE *fp = fopen(filename, "rb");
        if (!fp) return FALSE;
        char tmp[1 << 16];
        size_t r;
        while ((r = fread(tmp, 1, sizeof tmp, fp)) > 0) buf.append(tmp, r);
        fclose(fp);
    }
    if (buf.size() < 16 || memcmp(buf.data(), STATE_MAGIC, 8)) {
        NN_ERROR(stderr, "%s is not a libhpnn state file\n", filename);
        return FALSE;
    }
    UINT64 h;
    memcpy(&h, buf.data() + buf.size() - 8, 8);
    if (hpnn_fnv1a(buf.data(), buf.size() - 8, HPNN_FNV_SEED) != h) {
        NN_ERROR(stderr, "state file %s: checksum mismatch (truncated or corrupted)\n", filename);
        return FALSE;
    }
    Reader r(buf);
    char magic[8];
    r.get(magic, 8);
    const UINT type = r.u32(), train = r.u32(), L = r.u32(), has_mom = r.u32();
    (void)train;
    if (!r.ok || L != k->n_hiddens + 1 || type != (UINT)conf->type) {
        NN_ERROR(stderr, "state file %s does not match the network (layers / type)\n", filename);
        return FALSE;
    }
    std::vector<UINT> dims(L + 1);
    for (UINT i = 0; i <= L; i++) dims[i] = r.u32();
    bool match = r.ok && dims[0] == k->n_inputs;
    for (UINT l = 0; l < L && match; l++) match = dims[l + 1] == layer_at(k, l)->n_neurons;
    if (!match) {
        NN_ERROR(stderr, "state file %s does not match the network dimensions\n", filename);
        return FALSE;
    }
    const UINT seed = r.u32(), epochs = r.u32();
    r.u32();
    r.u32();
    UINT64 seen = 0;
    r.get(&seen, 8);
    std::vector<std::vector<DOUBLE>> W(L), V(L);
    for (UINT l = 0; l < L; l++) {
        const layer_ann *ly = layer_at(k, l);
        W[l].resize((size_t)ly->n_neurons * ly->n_inputs);
        r.get(W[l].data(), W[l].size() * 8);
    }
    if (has_mom)
        for (UINT l = 0; l < L; l++) {
            V[l].resize(W[l].size());
            r.get(V[l].data(), V[l].size() * 8);
        }
    if (!r.ok || r.off != buf.size() - 8) {
        NN_ERROR(stderr, "state file %s: bad size\n", filename);
        return FALSE;
    }
    for (UINT l = 0; l < L; l++) memcpy(layer_at(k, l)->weights, W[l].data(), W[l].size() * 8);
    if (has_mom) {
        ann_momentum_init(k);
        for (UINT l = 0; l < L; l++) memcpy(k->dw[l], V[l].data(), V[l].size() * 8);
    }
    hpnn_gpu_mark_host_dirty(k);
    conf->seed = seed;
    conf->epochs_done = epochs;
    conf->samples_seen = seen;
    conf->resume = has_mom ? TRUE : FALSE;
    NN_OUT(stdout, "state %s loaded: %u epochs done, %llu samples seen%s\n", filename, epochs,
           (unsigned long long)seen, has_mom ? ", momentum restored" : "");
    return TRUE;
}

extern "C" UINT _NN(return, epochs_done)(nn_def *conf) { return conf ? conf->epochs_done : 0; }
