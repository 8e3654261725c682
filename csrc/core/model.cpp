/*
 * libhpnn model definition: allocation, seeded generation, kernel.opt
 * reader/writer.
 *
 * Parity:
 *   - allocation / max_index      reference ann.c:113-202
 *   - generation                  reference ann.c:632-766: srandom(seed),
 *     w = 2(random()/RAND_MAX - 0.5)/sqrt(M), hidden layers first then the
 *     output layer, row-major -> bit-identical initial weights for a seed;
 *   - kernel.opt grammar          reference ann.c:770-857 (writer) and
 *     ann.c:206-631 (reader), see docs/FORMATS.md.  The reader here is a
 *     single-pass tokenizer that tolerates wrapped weight lines and files
 *     without a [param] line (dimensions are then taken from the block
 *     headers), and it loads the whole file before any device transfer
 *     (the reference copied every neuron row to the GPU separately,
 *     ann.c:445-448).
 */
#include <libhpnn/ann.h>
#include <math.h>
#include <string.h>
#include <time.h>
#include <ctype.h>
#include <vector>
#include <string>

#include "runtime_internal.h"

extern "C" kernel_ann *ann_kernel_allocate(UINT n_inputs, UINT n_hiddens, const UINT *hiddens,
                                           UINT n_outputs) {
    if (n_inputs == 0 || n_outputs == 0) return NULL;
    for (UINT i = 0; i < n_hiddens; i++)
        if (hiddens[i] == 0) return NULL;
    kernel_ann *k = (kernel_ann *)calloc(1, sizeof(kernel_ann));
    k->n_inputs = n_inputs;
    k->n_hiddens = n_hiddens;
    k->n_outputs = n_outputs;
    k->in = (DOUBLE *)calloc(n_inputs, sizeof(DOUBLE));
    k->hiddens = n_hiddens ? (layer_ann *)calloc(n_hiddens, sizeof(layer_ann)) : NULL;
    UINT prev = n_inputs, mx = n_inputs > n_outputs ? n_inputs : n_outputs;
    for (UINT i = 0; i < n_hiddens; i++) {
        layer_ann *l = &k->hiddens[i];
        l->n_neurons = hiddens[i];
        l->n_inputs = prev;
        l->weights = (DOUBLE *)calloc((size_t)l->n_neurons * l->n_inputs, sizeof(DOUBLE));
        l->vec = (DOUBLE *)calloc(l->n_neurons, sizeof(DOUBLE));
        prev = hiddens[i];
        if (hiddens[i] > mx) mx = hiddens[i];
    }
    k->output.n_neurons = n_outputs;
    k->output.n_inputs = prev;
    k->output.weights = (DOUBLE *)calloc((size_t)n_outputs * prev, sizeof(DOUBLE));
    k->output.vec = (DOUBLE *)calloc(n_outputs, sizeof(DOUBLE));
    k->max_index = mx;
    k->tmp_cpu = (DOUBLE *)calloc(mx, sizeof(DOUBLE));
    k->dw = NULL;
    k->gpu = NULL;
    return k;
}

/* the GPU engine registers a destructor for its per-kernel state */
void (*hpnn_gpu_model_destroy_hook)(kernel_ann *) = NULL;

extern "C" void ann_kernel_free(kernel_ann *k) {
    if (!k) return;
    if (k->gpu && hpnn_gpu_model_destroy_hook) hpnn_gpu_model_destroy_hook(k);
    ann_momentum_free(k);
    for (UINT i = 0; i < k->n_hiddens; i++) {
        free(k->hiddens[i].weights);
        free(k->hiddens[i].vec);
    }
    free(k->hiddens);
    free(k->output.weights);
    free(k->output.vec);
    free(k->in);
    free(k->tmp_cpu);
    free(k->name);
    free(k);
}

extern "C" UINT64 ann_n_params(const kernel_ann *k) {
    UINT64 p = 0;
    for (UINT i = 0; i < k->n_hiddens; i++) p += (UINT64)k->hiddens[i].n_neurons * k->hiddens[i].n_inputs;
    p += (UINT64)k->output.n_neurons * k->output.n_inputs;
    return p;
}

extern "C" kernel_ann *ann_generate(UINT *seed, UINT n_inputs, UINT n_hiddens, UINT n_outputs,
                                    const UINT *hiddens) {
    if (*seed == 0) *seed = (UINT)time(NULL);
    srandom(*seed);
    kernel_ann *k = ann_kernel_allocate(n_inputs, n_hiddens, hiddens, n_outputs);
    if (!k) return NULL;
    auto fill = [](layer_ann *l) {
        const DOUBLE scale = 1.0 / sqrt((DOUBLE)l->n_inputs);
        const size_t n = (size_t)l->n_neurons * l->n_inputs;
        for (size_t j = 0; j < n; j++) {
            DOUBLE r = (DOUBLE)random() / RAND_MAX;
            l->weights[j] = 2.0 * (r - 0.5) * scale;
        }
    };
    for (UINT i = 0; i < n_hiddens; i++) fill(&k->hiddens[i]);
    fill(&k->output);
    return k;
}

extern "C" BOOL ann_validate_kernel(const kernel_ann *k) {
    if (!k) return FALSE;
    if (k->n_inputs == 0 || k->n_outputs == 0) return FALSE;
    if (!k->in || !k->output.weights || !k->output.vec) return FALSE;
    for (UINT i = 0; i < k->n_hiddens; i++)
        if (!k->hiddens[i].weights || !k->hiddens[i].vec || k->hiddens[i].n_neurons == 0) return FALSE;
    return TRUE;
}

/* ------------------------------------------------------------------ */
/* kernel.opt writer                                                   */
/* ------------------------------------------------------------------ */
static void dump_layer(FILE *out, const layer_ann *l, const char *fmt_first, const char *fmt) {
    for (UINT j = 0; j < l->n_neurons; j++) {
        fprintf(out, "[neuron %u] %u\n", j + 1, l->n_inputs);
        const DOUBLE *row = l->weights + _2D_IDX(l->n_inputs, j, 0);
        fprintf(out, fmt_first, row[0]);
        for (UINT i = 1; i < l->n_inputs; i++) fprintf(out, fmt, row[i]);
        fputc('\n', out);
    }
}

extern "C" void ann_dump(const kernel_ann *k, FILE *out, BOOL exact) {
    if (!k) {
        NN_ERROR(stderr, "CAN'T SAVE KERNEL! kernel=NULL\n");
        return;
    }
    if (hpnn_output_rank() != 0) return;
    const char *f1 = exact ? "%.17g" : "%17.15f";
    const char *f2 = exact ? " %.17g" : " %17.15f";
    fprintf(out, "[name] %s\n", k->name ? k->name : "noname");
    fprintf(out, "[param] %u", k->n_inputs);
    for (UINT i = 0; i < k->n_hiddens; i++) fprintf(out, " %u", k->hiddens[i].n_neurons);
    fprintf(out, " %u\n", k->output.n_neurons);
    fprintf(out, "[input] %u\n", k->n_inputs);
    for (UINT i = 0; i < k->n_hiddens; i++) {
        fprintf(out, "[hidden %u] %u\n", i + 1, k->hiddens[i].n_neurons);
        dump_layer(out, &k->hiddens[i], f1, f2);
    }
    fprintf(out, "[output] %u\n", k->output.n_neurons);
    dump_layer(out, &k->output, f1, f2);
    fflush(out);
}

/* ------------------------------------------------------------------ */
/* kernel.opt reader                                                   */
/* ------------------------------------------------------------------ */
char *hpnn_readline(FILE *fp, char **buf, size_t *cap) {
    if (*buf == NULL || *cap == 0) {
        *cap = 4096;
        *buf = (char *)malloc(*cap);
    }
    size_t len = 0;
    for (;;) {
        if (!fgets(*buf + len, (int)(*cap - len), fp)) {
            if (len == 0) return NULL;
            break;
        }
        len += strlen(*buf + len);
        if (len > 0 && (*buf)[len - 1] == '\n') break;
        if (len + 1 >= *cap) {
            *cap *= 2;
            *buf = (char *)realloc(*buf, *cap);
        }
    }
    return *buf;
}

namespace {
struct Block {
    bool is_output;
    UINT index;     /* 1-based hidden index */
    UINT n_neurons;
};

/* parse "[tag N] value" or "[tag] value": returns pointer after ']' */
const char *after_bracket(const char *p) {
    const char *q = strchr(p, ']');
    return q ? q + 1 : NULL;
}

bool read_uint(const char *p, UINT *v) {
    while (*p && isspace((unsigned char)*p)) p++;
    if (!isdigit((unsigned char)*p)) return false;
    *v = (UINT)strtoul(p, NULL, 10);
    return true;
}
}  // namespace

extern "C" kernel_ann *ann_load(const CHAR *filename) {
    FILE *fp = fopen(filename, "r");
    if (!fp) {
        NN_ERROR(stderr, "Error opening kernel file: %s\n", filename);
        return NULL;
    }
    char *buf = NULL;
    size_t cap = 0;
    std::string name;
    std::vector<UINT> param;
    UINT n_in = 0;
    std::vector<Block> blocks;
    /* pass 1: headers only */
    while (hpnn_readline(fp, &buf, &cap)) {
        const char *p = buf;
        while (*p && isspace((unsigned char)*p)) p++;
        if (*p != '[') continue;
        if (!strncmp(p, "[name", 5)) {
            const char *q = after_bracket(p);
            if (q) {
                while (*q == ' ' || *q == '\t') q++;
                name.assign(q);
                while (!name.empty() && (name.back() == '\n' || name.back() == '\r' || name.back() == ' '))
                    name.pop_back();
            }
        } else if (!strncmp(p, "[param", 6)) {
            const char *q = after_bracket(p);
            char *e;
            while (q && *q) {
                while (*q && isspace((unsigned char)*q)) q++;
                if (!isdigit((unsigned char)*q)) break;
                param.push_back((UINT)strtoul(q, &e, 10));
                q = e;
            }
        } else if (!strncmp(p, "[input", 6)) {
            const char *q = after_bracket(p);
            if (q) read_uint(q, &n_in);
        } else if (!strncmp(p, "[hidden", 7)) {
            Block b{false, 0, 0};
            read_uint(p + 7, &b.index);
            const char *q = after_bracket(p);
            if (!q || !read_uint(q, &b.n_neurons)) goto fail_fmt;
            blocks.push_back(b);
        } else if (!strncmp(p, "[output", 7)) {
            Block b{true, 0, 0};
            const char *q = after_bracket(p);
            if (!q || !read_uint(q, &b.n_neurons)) goto fail_fmt;
            blocks.push_back(b);
        }
    }
    {
        if (blocks.empty() || !blocks.back().is_output) goto fail_fmt;
        std::vector<UINT> hid;
        for (size_t i = 0; i + 1 < blocks.size(); i++) {
            if (blocks[i].is_output) goto fail_fmt;
            hid.push_back(blocks[i].n_neurons);
        }
        UINT n_out = blocks.back().n_neurons;
        if (n_in == 0 && !param.empty()) n_in = param[0];
        if (!param.empty()) {
            /* [param] must agree with the block headers */
            if (param.size() != hid.size() + 2 || param[0] != n_in || param.back() != n_out) goto fail_fmt;
            for (size_t i = 0; i < hid.size(); i++)
                if (param[i + 1] != hid[i]) goto fail_fmt;
        }
        kernel_ann *k = ann_kernel_allocate(n_in, (UINT)hid.size(), hid.data(), n_out);
        if (!k) goto fail_fmt;
        k->name = strdup(name.empty() ? "noname" : name.c_str());
        /* pass 2: weights */
        rewind(fp);
        layer_ann *cur = NULL;
        UINT hidden_seen = 0;
        UINT row = 0;
        size_t filled = 0;   /* values filled in the current row */
        bool in_row = false;
        while (hpnn_readline(fp, &buf, &cap)) {
            const char *p = buf;
            while (*p && isspace((unsigned char)*p)) p++;
            if (*p == '[') {
                if (in_row && filled != cur->n_inputs) goto fail_k;
                in_row = false;
                if (!strncmp(p, "[hidden", 7)) {
                    cur = &k->hiddens[hidden_seen++];
                    row = 0;
                } else if (!strncmp(p, "[output", 7)) {
                    cur = &k->output;
                    row = 0;
                } else if (!strncmp(p, "[neuron", 7)) {
                    if (!cur) goto fail_k;
                    UINT idx = 0, m = 0;
                    read_uint(p + 7, &idx);
                    const char *q = after_bracket(p);
                    if (!q || !read_uint(q, &m) || m != cur->n_inputs) goto fail_k;
                    row = idx ? idx - 1 : row;
                    if (row >= cur->n_neurons) goto fail_k;
                    in_row = true;
                    filled = 0;
                }
                continue;
            }
            if (!in_row) continue;
            char *e;
            const char *q = p;
            DOUBLE *dst = cur->weights + _2D_IDX(cur->n_inputs, row, 0);
            while (*q && filled < cur->n_inputs) {
                DOUBLE v = strtod(q, &e);
                if (e == q) break;
                dst[filled++] = v;
                q = e;
            }
            if (filled == cur->n_inputs) {
                in_row = false;
                row++;
            }
        }
        if (in_row) goto fail_k;
        free(buf);
        fclose(fp);
        return k;
    fail_k:
        ann_kernel_free(k);
        NN_ERROR(stderr, "kernel file %s: malformed weights\n", filename);
        free(buf);
        fclose(fp);
        return NULL;
    }
fail_fmt:
    NN_ERROR(stderr, "kernel file %s: malformed header\n", filename);
    free(buf);
    fclose(fp);
    return NULL;
}
