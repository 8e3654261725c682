/*
 * libhpnn C API: configuration, kernel management, sample I/O and the
 * train / run workflows.
 *
 * Parity map (reference src/libhpnn.c):
 *   conf setters/getters          :544-657
 *   nn_load_conf / nn_dump_conf   :658-937  (same keys; values are read
 *                                  after the closing ']' so both "[input]"
 *                                  and the dumped "[inputs]" parse)
 *   kernel generate/load/dump     :941-1009
 *   accessors                     :1013-1066 (work for generated kernels
 *                                  too; the reference returned 0 there)
 *   nn_read_sample                :1070-1145
 *   nn_train_kernel               :1149-1302 (same file walk, same seeded
 *                                  permutation, same log lines; the file
 *                                  list is sorted first so the order does
 *                                  not depend on readdir, and the
 *                                  random()*n/RAND_MAX == n overflow is
 *                                  rejected instead of indexing past the end)
 *   nn_run_kernel                 :1306-1536
 * Extensions: [mode] online|batched, [dtype], [device], [batch], [epochs],
 * [lr], [momentum] conf keys; batched training on CPU (FP64) or GPU.
 */
#include <libhpnn/ann.h>
#include <ctype.h>
#include <dirent.h>
#include <math.h>
#include <stdarg.h>
#include <string.h>
#include <time.h>
#include <algorithm>
#include <string>
#include <vector>

#include <libhpnn/observe.h>
#include <omp.h>

#include "dataset.h"
#include "runtime_internal.h"
#include "../gpu/engine.h"

#define KERN(conf) ((kernel_ann *)((conf)->kernel))

static UINT g_last_pass = 0, g_last_total = 0;

/* ------------------------------------------------------------------ */
/* configuration                                                       */
/* ------------------------------------------------------------------ */
extern "C" void _NN(init, conf)(nn_def *conf) {
    memset(conf, 0, sizeof(*conf));
    conf->rr = hpnn_rt_get();
    conf->type = NN_TYPE_UKN;
    conf->train = NN_TRAIN_UKN;
    conf->need_init = FALSE;
    conf->seed = 0;
    conf->mode = NN_MODE_ONLINE;
    conf->dtype = NN_DTYPE_F64;
    conf->device = NN_DEVICE_AUTO;
    conf->batch = 256;
    conf->epochs = 1;
    conf->lr = -1.0;
    conf->momentum = -1.0;
}

extern "C" void _NN(free, kernel)(nn_def *conf) {
    if (!conf || !conf->kernel) return;
    ann_kernel_free(KERN(conf));
    conf->kernel = NULL;
}

extern "C" void _NN(deinit, conf)(nn_def *conf) {
    if (!conf) return;
    _NN(free, kernel)(conf);
    free(conf->name);
    free(conf->f_kernel);
    free(conf->samples);
    free(conf->tests);
    conf->name = conf->f_kernel = conf->samples = conf->tests = NULL;
}

static void set_str(CHAR **dst, const CHAR *src) {
    free(*dst);
    *dst = src ? strdup(src) : NULL;
}

extern "C" void _NN(set, name)(nn_def *c, const CHAR *n) {
    set_str(&c->name, n);
    if (c->kernel) set_str(&KERN(c)->name, n);
}
extern "C" void _NN(get, name)(nn_def *c, CHAR **n) { *n = c->name ? strdup(c->name) : NULL; }
extern "C" char *_NN(return, name)(nn_def *c) { return c->name; }
extern "C" void _NN(set, type)(nn_def *c, nn_type t) { c->type = t; }
extern "C" void _NN(get, type)(nn_def *c, nn_type *t) { *t = c->type; }
extern "C" nn_type _NN(return, type)(nn_def *c) { return c->type; }
extern "C" void _NN(set, need_init)(nn_def *c, BOOL v) { c->need_init = v; }
extern "C" void _NN(get, need_init)(nn_def *c, BOOL *v) { *v = c->need_init; }
extern "C" BOOL _NN(return, need_init)(nn_def *c) { return c->need_init; }
extern "C" void _NN(set, seed)(nn_def *c, UINT s) { c->seed = s; }
extern "C" void _NN(get, seed)(nn_def *c, UINT *s) { *s = c->seed; }
extern "C" UINT _NN(return, seed)(nn_def *c) { return c->seed; }
extern "C" void _NN(set, kernel_filename)(nn_def *c, CHAR *f) { set_str(&c->f_kernel, f); }
extern "C" void _NN(get, kernel_filename)(nn_def *c, CHAR **f) { *f = c->f_kernel ? strdup(c->f_kernel) : NULL; }
extern "C" char *_NN(return, kernel_filename)(nn_def *c) { return c->f_kernel; }
extern "C" void _NN(set, train)(nn_def *c, nn_train t) { c->train = t; }
extern "C" void _NN(get, train)(nn_def *c, nn_train *t) { *t = c->train; }
extern "C" nn_train _NN(return, train)(nn_def *c) { return c->train; }
extern "C" void _NN(set, samples_directory)(nn_def *c, CHAR *s) { set_str(&c->samples, s); }
extern "C" void _NN(get, samples_directory)(nn_def *c, CHAR **s) { *s = c->samples ? strdup(c->samples) : NULL; }
extern "C" char *_NN(return, samples_directory)(nn_def *c) { return c->samples; }
extern "C" void _NN(set, tests_directory)(nn_def *c, CHAR *s) { set_str(&c->tests, s); }
extern "C" void _NN(get, tests_directory)(nn_def *c, CHAR **s) { *s = c->tests ? strdup(c->tests) : NULL; }
extern "C" char *_NN(return, tests_directory)(nn_def *c) { return c->tests; }
extern "C" void _NN(set, mode)(nn_def *c, nn_mode m) { c->mode = m; }
extern "C" nn_mode _NN(return, mode)(nn_def *c) { return c->mode; }
extern "C" void _NN(set, dtype)(nn_def *c, nn_dtype d) { c->dtype = d; }
extern "C" nn_dtype _NN(return, dtype)(nn_def *c) { return c->dtype; }
extern "C" void _NN(set, device)(nn_def *c, nn_device d) { c->device = d; }
extern "C" nn_device _NN(return, device)(nn_def *c) { return c->device; }
extern "C" void _NN(set, batch)(nn_def *c, UINT b) { c->batch = b ? b : 1; }
extern "C" UINT _NN(return, batch)(nn_def *c) { return c->batch; }
extern "C" void _NN(set, epochs)(nn_def *c, UINT e) { c->epochs = e ? e : 1; }
extern "C" UINT _NN(return, epochs)(nn_def *c) { return c->epochs; }
extern "C" void _NN(set, learning_rate)(nn_def *c, DOUBLE lr) { c->lr = lr; }
extern "C" DOUBLE _NN(return, learning_rate)(nn_def *c) { return c->lr; }
extern "C" void _NN(set, momentum)(nn_def *c, DOUBLE a) { c->momentum = a; }
extern "C" DOUBLE _NN(return, momentum)(nn_def *c) { return c->momentum; }
extern "C" UINT _NN(return, last_pass)(void) { return g_last_pass; }
extern "C" UINT _NN(return, last_total)(void) { return g_last_total; }

/* ---- conf parsing helpers ---- */
static std::string trim(const std::string &s) {
    size_t a = 0, b = s.size();
    while (a < b && isspace((unsigned char)s[a])) a++;
    while (b > a && isspace((unsigned char)s[b - 1])) b--;
    return s.substr(a, b - a);
}
/* strip a trailing '#' comment */
static std::string value_of(const char *after) {
    std::string v(after);
    size_t h = v.find('#');
    if (h != std::string::npos) v = v.substr(0, h);
    return trim(v);
}

static bool parse_uint_list(const std::string &v, std::vector<UINT> &out) {
    const char *p = v.c_str();
    char *e;
    out.clear();
    while (*p) {
        while (*p && isspace((unsigned char)*p)) p++;
        if (!*p) break;
        if (!isdigit((unsigned char)*p)) return false;
        out.push_back((UINT)strtoul(p, &e, 10));
        p = e;
    }
    return !out.empty();
}

extern "C" nn_def *_NN(load, conf)(const CHAR *filename) {
    nn_def *conf = (nn_def *)calloc(1, sizeof(nn_def));
    _NN(init, conf)(conf);
    UINT n_in = 0, n_out = 0;
    std::vector<UINT> hid;
    FILE *fp = fopen(filename, "r");
    char *buf = NULL;
    size_t cap = 0;
    if (!fp) {
        NN_ERROR(stderr, "Error opening configuration file: %s\n", filename);
        free(conf);
        return NULL;
    }
#define CONF_FAIL(...)                                                     \
    do {                                                                   \
        NN_ERROR(stderr, "Malformed NN configuration file!\n");            \
        NN_ERROR(stderr, __VA_ARGS__);                                     \
        goto fail;                                                         \
    } while (0)
    while (hpnn_readline(fp, &buf, &cap)) {
        const char *lb = strchr(buf, '[');
        if (!lb) continue;
        const char *rb = strchr(lb, ']');
        if (!rb) continue;
        std::string key(lb + 1, rb - lb - 1);
        std::string v = value_of(rb + 1);
        auto is = [&](const char *k) { return key.compare(0, strlen(k), k) == 0; };
        if (is("name")) {
            set_str(&conf->name, v.c_str());
        } else if (is("type")) {
            switch (v.empty() ? 'A' : toupper(v[0])) {
                case 'L': conf->type = NN_TYPE_LNN; break;
                case 'S': conf->type = NN_TYPE_SNN; break;
                default: conf->type = NN_TYPE_ANN; break;
            }
        } else if (is("init")) {
            if (v.find("generate") != std::string::npos || v.find("GENERATE") != std::string::npos) {
                NN_OUT(stdout, "generating kernel!\n");
                conf->need_init = TRUE;
            } else {
                NN_OUT(stdout, "loading kernel!\n");
                conf->need_init = FALSE;
                if (v.empty()) CONF_FAIL("[init] can't read filename: %s\n", buf);
                set_str(&conf->f_kernel, v.c_str());
            }
        } else if (is("seed")) {
            if (v.empty() || !isdigit((unsigned char)v[0])) CONF_FAIL("[seed] value: %s\n", v.c_str());
            conf->seed = (UINT)strtoul(v.c_str(), NULL, 10);
        } else if (is("input")) {
            if (v.empty() || !isdigit((unsigned char)v[0])) CONF_FAIL("[input] value: %s\n", v.c_str());
            n_in = (UINT)strtoul(v.c_str(), NULL, 10);
        } else if (is("hidden")) {
            if (!parse_uint_list(v, hid)) CONF_FAIL("[hidden] value: %s\n", v.c_str());
        } else if (is("output")) {
            if (v.empty() || !isdigit((unsigned char)v[0])) CONF_FAIL("[output] value: %s\n", v.c_str());
            n_out = (UINT)strtoul(v.c_str(), NULL, 10);
        } else if (is("train")) {
            std::string u = v;
            for (auto &ch : u) ch = (char)toupper(ch);
            if (!u.empty() && u[0] == 'B') conf->train = (u.size() > 2 && u[2] == 'M') ? NN_TRAIN_BPM : NN_TRAIN_BP;
            else if (!u.empty() && u[0] == 'C') conf->train = NN_TRAIN_CG;
            else if (!u.empty() && u[0] == 'S') conf->train = NN_TRAIN_SPLX;
            else conf->train = NN_TRAIN_UKN;
        } else if (is("sample_dir") || is("samples")) {
            set_str(&conf->samples, v.c_str());
        } else if (is("test_dir") || is("tests")) {
            set_str(&conf->tests, v.c_str());
        } else if (is("mode")) {
            conf->mode = (!v.empty() && toupper(v[0]) == 'B') ? NN_MODE_BATCHED : NN_MODE_ONLINE;
        } else if (is("dtype")) {
            std::string u = v;
            for (auto &ch : u) ch = (char)tolower(ch);
            if (u == "bf16") conf->dtype = NN_DTYPE_BF16;
            else if (u == "f32" || u == "fp32" || u == "float") conf->dtype = NN_DTYPE_F32;
            else if (u == "f64" || u == "fp64" || u == "double") conf->dtype = NN_DTYPE_F64;
            else CONF_FAIL("[dtype] unknown: %s (f64 | f32 | bf16)\n", v.c_str()); /* docs/PARITY.md */
        } else if (is("device")) {
            std::string u = v;
            for (auto &ch : u) ch = (char)tolower(ch);
            conf->device = u == "cpu" ? NN_DEVICE_CPU : (u == "gpu" ? NN_DEVICE_GPU : NN_DEVICE_AUTO);
        } else if (is("batch")) {
            conf->batch = (UINT)strtoul(v.c_str(), NULL, 10);
            if (!conf->batch) conf->batch = 1;
        } else if (is("epochs")) {
            conf->epochs = (UINT)strtoul(v.c_str(), NULL, 10);
            if (!conf->epochs) conf->epochs = 1;
        } else if (is("parallel")) {
            std::string u = v;
            for (auto &ch : u) ch = (char)tolower(ch);
            conf->parallel = u == "tp" ? NN_PARALLEL_TP : NN_PARALLEL_DP;
        } else if (is("lr")) {
            conf->lr = strtod(v.c_str(), NULL);
        } else if (is("momentum")) {
            conf->momentum = strtod(v.c_str(), NULL);
        }
    }
    fclose(fp);
    fp = NULL;
    if (conf->type == NN_TYPE_UKN) CONF_FAIL("[type] unknown or missing...\n");
    if (conf->need_init) {
        if (n_in == 0) CONF_FAIL("[input] wrong or missing...\n");
        if (hid.empty()) CONF_FAIL("[hidden] wrong or missing...\n");
        if (n_out == 0) CONF_FAIL("[output] wrong or missing...\n");
        for (UINT h : hid)
            if (h == 0) CONF_FAIL("[hidden] some have a 0 neuron content!\n");
        if (!_NN(generate, kernel)(conf, n_in, (UINT)hid.size(), n_out, hid.data())) {
            NN_ERROR(stderr, "FAILED to generate NN kernel!\n");
            goto fail;
        }
    } else {
        if (!_NN(load, kernel)(conf)) {
            NN_ERROR(stderr, "FAILED to load the NN kernel!\n");
            goto fail;
        }
    }
    free(buf);
    return conf;
fail:
#undef CONF_FAIL
    if (fp) fclose(fp);
    free(buf);
    _NN(deinit, conf)(conf);
    free(conf);
    return NULL;
}

extern "C" void _NN(dump, conf)(nn_def *conf, FILE *fp) {
    if (!conf) return;
    static const char *tn[] = {"ANN", "LNN", "SNN"};
    static const char *trn[] = {"BP", "BPM", "CG", "SPLX"};
    _OUT(fp, "# NN configuration (libhpnn-mi355x)\n");
    _OUT(fp, "[name] %s\n", conf->name ? conf->name : "noname");
    _OUT(fp, "[type] %s\n", (conf->type >= 0 && conf->type <= 2) ? tn[conf->type] : "UKN");
    if (conf->need_init || !conf->f_kernel) _OUT(fp, "[init] generate\n");
    else _OUT(fp, "[init] %s\n", conf->f_kernel);
    _OUT(fp, "[seed] %u\n", conf->seed);
    kernel_ann *k = KERN(conf);
    if (k) {
        _OUT(fp, "[inputs] %u\n", k->n_inputs);
        _OUT(fp, "[hiddens]");
        for (UINT i = 0; i < k->n_hiddens; i++) _OUT(fp, " %u", k->hiddens[i].n_neurons);
        _OUT(fp, "\n[outputs] %u\n", k->n_outputs);
    }
    _OUT(fp, "[train] %s\n", (conf->train >= 0 && conf->train <= 3) ? trn[conf->train] : "UKN");
    if (conf->samples) _OUT(fp, "[sample_dir] %s\n", conf->samples);
    if (conf->tests) _OUT(fp, "[test_dir] %s\n", conf->tests);
    if (conf->mode == NN_MODE_BATCHED) {
        static const char *dn[] = {"f64", "f32", "bf16"};
        _OUT(fp, "[mode] batched\n[batch] %u\n[epochs] %u\n[dtype] %s\n", conf->batch, conf->epochs,
             dn[conf->dtype]);
        if (conf->parallel == NN_PARALLEL_TP) _OUT(fp, "[parallel] tp\n");
    }
    if (conf->lr > 0) _OUT(fp, "[lr] %.17g\n", conf->lr);
    if (conf->momentum >= 0) _OUT(fp, "[momentum] %.17g\n", conf->momentum);
}

/* ------------------------------------------------------------------ */
/* kernel management                                                   */
/* ------------------------------------------------------------------ */
extern "C" BOOL _NN(generate, kernel)(nn_def *conf, ...) {
    va_list ap;
    va_start(ap, conf);
    UINT n_in = va_arg(ap, UINT);
    UINT n_hid = va_arg(ap, UINT);
    UINT n_out = va_arg(ap, UINT);
    UINT *hiddens = va_arg(ap, UINT *);
    va_end(ap);
    if (conf->type == NN_TYPE_UKN) return FALSE;
    _NN(free, kernel)(conf);
    kernel_ann *k = ann_generate(&conf->seed, n_in, n_hid, n_out, hiddens);
    if (!k) return FALSE;
    k->name = strdup(conf->name ? conf->name : "noname");
    conf->kernel = k;
    conf->need_init = TRUE;
    NN_OUT(stdout, "generated kernel: %llu parameters\n", (unsigned long long)ann_n_params(k));
    return TRUE;
}

extern "C" BOOL _NN(load, kernel)(nn_def *conf) {
    if (!conf->f_kernel) return FALSE;
    if (conf->type == NN_TYPE_UKN) return FALSE;
    _NN(free, kernel)(conf);
    kernel_ann *k = ann_load(conf->f_kernel);
    if (!k) return FALSE;
    if (conf->name) {
        free(k->name);
        k->name = strdup(conf->name);
    } else {
        conf->name = strdup(k->name);
    }
    conf->kernel = k;
    return TRUE;
}

extern "C" void _NN(dump, kernel)(nn_def *conf, FILE *out) {
    if (!conf || !conf->kernel) {
        NN_ERROR(stderr, "CAN'T SAVE KERNEL! kernel=NULL\n");
        return;
    }
    hpnn_gpu_sync_host(KERN(conf));
    ann_dump(KERN(conf), out, FALSE);
}

extern "C" void _NN(dump, kernel_exact)(nn_def *conf, FILE *out) {
    if (!conf || !conf->kernel) return;
    hpnn_gpu_sync_host(KERN(conf));
    ann_dump(KERN(conf), out, TRUE);
}

extern "C" UINT _NN(get, n_inputs)(nn_def *c) { return c && c->kernel ? KERN(c)->n_inputs : 0; }
extern "C" UINT _NN(get, n_hiddens)(nn_def *c) { return c && c->kernel ? KERN(c)->n_hiddens : 0; }
extern "C" UINT _NN(get, n_outputs)(nn_def *c) { return c && c->kernel ? KERN(c)->n_outputs : 0; }
extern "C" UINT _NN(get, h_neurons)(nn_def *c, UINT layer) {
    if (!c || !c->kernel || layer >= KERN(c)->n_hiddens) return 0;
    return KERN(c)->hiddens[layer].n_neurons;
}

/* ------------------------------------------------------------------ */
/* samples                                                             */
/* ------------------------------------------------------------------ */
static bool read_vector(FILE *fp, char **buf, size_t *cap, UINT n, DOUBLE *dst) {
    UINT got = 0;
    while (got < n && hpnn_readline(fp, buf, cap)) {
        const char *p = *buf;
        char *e;
        while (got < n) {
            DOUBLE v = strtod(p, &e);
            if (e == p) break;
            dst[got++] = v;
            p = e;
        }
        if (got < n) {
            /* values may be wrapped: continue only if the line was numeric */
            const char *q = p;
            while (*q && isspace((unsigned char)*q)) q++;
            if (*q) break;
        }
    }
    return got == n;
}

extern "C" BOOL _NN(read, sample)(CHAR *filename, DOUBLE **in, DOUBLE **out) {
    *in = NULL;
    *out = NULL;
    if (!filename) return FALSE;
    FILE *fp = fopen(filename, "r");
    if (!fp) return FALSE;
    char *buf = NULL;
    size_t cap = 0;
    BOOL ok = TRUE;
    while (ok && hpnn_readline(fp, &buf, &cap)) {
        const char *p = strchr(buf, '[');
        if (!p) continue;
        bool is_in = !strncmp(p, "[input", 6), is_out = !strncmp(p, "[output", 7);
        if (!is_in && !is_out) continue;
        const char *rb = strchr(p, ']');
        UINT n = 0;
        if (rb) {
            const char *q = rb + 1;
            while (*q && isspace((unsigned char)*q)) q++;
            if (isdigit((unsigned char)*q)) n = (UINT)strtoul(q, NULL, 10);
        }
        if (n == 0) {
            NN_ERROR(stderr, "sample %s %s read failed!\n", filename, is_in ? "input" : "output");
            ok = FALSE;
            break;
        }
        DOUBLE **dst = is_in ? in : out;
        free(*dst);
        *dst = (DOUBLE *)malloc(sizeof(DOUBLE) * n);
        if (!read_vector(fp, &buf, &cap, n, *dst)) {
            NN_ERROR(stderr, "sample %s %s read failed!\n", filename, is_in ? "input" : "output");
            ok = FALSE;
        }
    }
    fclose(fp);
    free(buf);
    if (!ok || !*in || !*out) {
        free(*in);
        free(*out);
        *in = *out = NULL;
        return FALSE;
    }
    return TRUE;
}

/* ------------------------------------------------------------------ */
/* workflow helpers                                                    */
/* ------------------------------------------------------------------ */
/* seeded permutation without replacement (reference libhpnn.c:1218-1229) */
static std::vector<UINT> seeded_order(UINT n, UINT seed) {
    srandom(seed);
    std::vector<UINT> order;
    std::vector<char> used(n, 0);
    order.reserve(n);
    for (UINT j = 0; j < n; j++) {
        UINT idx;
        do {
            idx = (UINT)((DOUBLE)random() * n / RAND_MAX);
        } while (idx >= n || used[idx]);
        used[idx] = 1;
        order.push_back(idx);
    }
    return order;
}

static bool use_gpu(const nn_def *conf) {
    if (conf->device == NN_DEVICE_CPU) return false;
    bool avail = hpnn_rt_gpu_available();
    if (conf->device == NN_DEVICE_GPU && !avail) {
        NN_ERROR(stderr, "GPU requested but no GPU available!\n");
    }
    return avail;
}

static DOUBLE default_lr(const nn_def *conf, bool gpu) {
    if (conf->lr > 0) return conf->lr;
    if (gpu || conf->mode == NN_MODE_BATCHED) return GPU_LEARN_RATE;
    if (conf->type == NN_TYPE_ANN) return conf->train == NN_TRAIN_BPM ? BPM_LEARN_RATE : BP_LEARN_RATE;
    return GPU_LEARN_RATE;
}

static DOUBLE default_alpha(const nn_def *conf) { return conf->momentum >= 0 ? conf->momentum : BPM_MOMENTUM; }

/* ------------------------------------------------------------------ */
/* training                                                            */
/* ------------------------------------------------------------------ */
extern "C" BOOL _NN(train, kernel)(nn_def *conf) {
    if (!conf || !conf->kernel || !conf->samples || conf->type == NN_TYPE_UKN) return FALSE;
    kernel_ann *k = KERN(conf);
    if (conf->train != NN_TRAIN_BP && conf->train != NN_TRAIN_BPM) {
        NN_ERROR(stdout, "unimplemented training type!\n");
        return FALSE;
    }
    HpnnTraceRange tr("nn_train_kernel");
    HpnnSamples src;
    if (!src.open(conf->samples)) {
        NN_ERROR(stderr, "can't open sample directory: %s\n", conf->samples);
        return FALSE;
    }
    if (conf->seed == 0) conf->seed = (UINT)time(NULL);
    const bool gpu = use_gpu(conf);
    const DOUBLE lr = default_lr(conf, gpu);
    const DOUBLE alpha = default_alpha(conf);

    if (conf->mode == NN_MODE_BATCHED) {
        std::vector<UINT> order = seeded_order((UINT)src.size(), conf->seed);
        std::vector<DOUBLE> X, T;
        UINT n;
        {
            HpnnTraceRange tl("load_samples");
            n = (UINT)src.load(order, k->n_inputs, k->n_outputs, _NN(return, omp_threads)(), X, T);
        }
        if (n == 0) return FALSE;
        hpnn_batched_opts o;
        memset(&o, 0, sizeof(o));
        o.type = conf->type;
        o.train = conf->train;
        o.dtype = conf->dtype;
        o.batch = conf->batch;
        o.epochs = conf->epochs;
        o.lr = lr;
        o.alpha = conf->train == NN_TRAIN_BPM ? alpha : 0.0;
        o.seed = conf->seed;
        o.resume = conf->resume && k->dw != NULL;
        o.epoch0 = conf->epochs_done;
        UINT ng = 1;
        _NN(get, n_gpu)(&ng);
        o.n_gpu = ng ? ng : 1;
        {
            const char *pe = getenv("HPNN_PARALLEL");
            o.tp = (pe ? (pe[0] == 't' || pe[0] == 'T') : conf->parallel == NN_PARALLEL_TP) ? 1 : 0;
        }
        hpnn_batched_stats st;
        memset(&st, 0, sizeof(st));
        BOOL ok;
        {
            HpnnTraceRange tb(gpu ? "train_batched_gpu" : "train_batched_cpu");
            ok = gpu ? hpnn_gpu_train_batched(k, X.data(), T.data(), n, &o, &st)
                     : hpnn_cpu_train_batched(k, X.data(), T.data(), n, &o, &st);
        }
        if (ok) {
            conf->epochs_done += conf->epochs;
            conf->samples_seen += st.samples;
        }
        NN_OUT(stdout, "BATCHED TRAINING: %llu samples in %.6f s (%.1f samples/s) loss=%.10f acc=%u/%u\n",
               (unsigned long long)st.samples, st.seconds, st.seconds > 0 ? st.samples / st.seconds : 0.0,
               st.epoch_loss, st.correct, n);
        if (hpnn_metrics_active()) {
            char buf[384];
            snprintf(buf, sizeof buf,
                     "\"engine\": \"%s\", \"ok\": %s, \"samples\": %llu, \"seconds\": %.6f, \"samples_per_s\": %.3f, "
                     "\"loss\": %.10g, \"correct\": %u, \"n\": %u, \"epochs_done\": %u",
                     gpu ? "gpu" : "cpu", ok ? "true" : "false", (unsigned long long)st.samples, st.seconds,
                     st.seconds > 0 ? st.samples / st.seconds : 0.0, st.epoch_loss, st.correct, n, conf->epochs_done);
            hpnn_metrics_emit("train_batched", buf);
        }
        return ok;
    }

    /* online (reference) mode */
    std::vector<UINT> order = seeded_order((UINT)src.size(), conf->seed);
    UINT n_ok = 0, n_done = 0;
    for (UINT idx : order) {
        const std::string &f = src.names[idx];
        NN_OUT(stdout, "TRAINING FILE: %16.16s\t", f.c_str());
        DOUBLE *in = NULL, *out = NULL;
        if (!src.get(idx, &in, &out)) continue;
        HpnnTraceRange ts("train_sample");
        UINT it = 0;
        BOOL ok = FALSE, first = FALSE;
        DOUBLE e0 = 0.0, r;
        if (gpu)
            r = hpnn_gpu_train_sample(k, conf->type, conf->train, in, out, lr, alpha, -1., &it, &ok, &e0, &first);
        else
            r = hpnn_cpu_train_sample(k, conf->type, conf->train, in, out, lr, alpha, -1., &it, &ok, &e0, &first);
        NN_COUT(stdout, " init=%15.10f", e0);
        NN_COUT(stdout, first ? " OK" : " NO");
        NN_COUT(stdout, " N_ITER=%8u", it);
        NN_COUT(stdout, " final=%15.10f", r);
        NN_COUT(stdout, ok ? " SUCCESS!\n" : " FAIL!\n");
        fflush(stdout);
        if (r > 0.1) NN_DBG(stdout, "bad optimization!\n");
        if (hpnn_metrics_active()) {
            char buf[384];
            snprintf(buf, sizeof buf,
                     "\"file\": \"%s\", \"init\": %.10g, \"first_ok\": %s, \"n_iter\": %u, \"final\": %.10g, "
                     "\"success\": %s",
                     f.c_str(), e0, first ? "true" : "false", it, r, ok ? "true" : "false");
            hpnn_metrics_emit("train_sample", buf);
        }
        n_ok += ok ? 1 : 0;
        n_done++;
        conf->samples_seen++;
        free(in);
        free(out);
        if (gpu && hpnn_gpu_failed(k)) {
            NN_ERROR(stderr, "GPU device state lost after %u samples: training aborted\n", n_done);
            return FALSE;
        }
    }
    if (gpu) hpnn_gpu_sync_host(k);
    if (hpnn_metrics_active()) {
        char buf[128];
        snprintf(buf, sizeof buf, "\"samples\": %u, \"success\": %u", n_done, n_ok);
        hpnn_metrics_emit("train_online", buf);
    }
    return TRUE;
}

/* ------------------------------------------------------------------ */
/* evaluation                                                          */
/* ------------------------------------------------------------------ */
extern "C" void _NN(run, kernel)(nn_def *conf) {
    g_last_pass = g_last_total = 0;
    if (!conf || !conf->kernel || !conf->tests || conf->type == NN_TYPE_UKN) return;
    kernel_ann *k = KERN(conf);
    HpnnSamples src;
    if (!src.open(conf->tests)) {
        NN_ERROR(stderr, "can't open test directory: %s\n", conf->tests);
        return;
    }
    HpnnTraceRange tr("nn_run_kernel");
    if (conf->seed == 0) conf->seed = (UINT)time(NULL);
    const bool gpu = use_gpu(conf);
    std::vector<UINT> order = seeded_order((UINT)src.size(), conf->seed);
    /* GPU: the whole test set goes through the batched engine of the model's precision
     * ([dtype], default f64 = the reference's) in one call -- one launch sequence and one
     * device-to-host copy per block of samples instead of one kernel launch, copy and host
     * sync per file; the per-file lines below are then produced from the outputs.
     * HPNN_RUN_ONLINE=1 keeps the reference's one-forward-per-file loop. */
    const char *ro = getenv("HPNN_RUN_ONLINE");
    const bool batched = gpu && !(ro && ro[0] == '1');
    std::vector<DOUBLE> Xall, Tall, Yall;
    std::vector<long> row_of(order.size(), -1);
    if (batched) {
        long rows = 0;
        for (size_t p = 0; p < order.size(); p++) {
            DOUBLE *in = NULL, *out = NULL;
            if (!src.get(order[p], &in, &out)) continue;
            Xall.insert(Xall.end(), in, in + k->n_inputs);
            Tall.insert(Tall.end(), out, out + k->n_outputs);
            row_of[p] = rows++;
            free(in);
            free(out);
        }
        Yall.assign((size_t)rows * k->n_outputs, 0.0);
        if (rows > 0 && !hpnn_gpu_infer_batched(k, conf->type, conf->dtype, Xall.data(), (UINT)rows, Yall.data())) {
            NN_ERROR(stderr, "batched GPU evaluation failed\n");
            return;
        }
    }
    for (size_t p = 0; p < order.size(); p++) {
        const UINT idx = order[p];
        const std::string &f = src.names[idx];
        NN_OUT(stdout, "TESTING FILE: %16.16s\t", f.c_str());
        DOUBLE *in = NULL, *out = NULL;
        const DOUBLE *o;
        if (batched) {
            if (row_of[p] < 0) continue;
            o = Yall.data() + (size_t)row_of[p] * k->n_outputs;
            out = Tall.data() + (size_t)row_of[p] * k->n_outputs;
        } else {
            if (!src.get(idx, &in, &out)) continue;
            if (gpu) {
                hpnn_gpu_forward(k, conf->type, in);
            } else {
                memcpy(k->in, in, sizeof(DOUBLE) * k->n_inputs);
                hpnn_cpu_forward(k, conf->type);
            }
            o = k->output.vec;
        }
        UINT guess, truth = 0;
        DOUBLE res;
        if (conf->type == NN_TYPE_ANN) {
            res = -1.;
            guess = k->n_outputs;
            truth = 0;
            for (UINT i = 0; i < k->n_outputs; i++) {
                if (res < o[i]) {
                    guess = i;
                    res = o[i];
                }
                if (out[i] > 0.5) truth = i;
            }
        } else {
            res = 0.;
            guess = 0;
            NN_DBG(stdout, " CLASS | PROBABILITY (%%)\n");
            NN_DBG(stdout, "-------|----------------\n");
            for (UINT i = 0; i < k->n_outputs; i++) {
                NN_DBG(stdout, " %5u | %15.10f\n", i + 1, o[i] * 100.);
                if (o[i] > res) {
                    res = o[i];
                    guess = i;
                }
                if (out[i] > 0.1) truth = i;
            }
            NN_DBG(stdout, "-------|----------------\n");
            NN_COUT(stdout, " BEST CLASS idx=%u P=%15.10f", guess + 1, res * 100);
        }
        g_last_total++;
        if (guess == truth) {
            g_last_pass++;
            NN_COUT(stdout, " [PASS]\n");
        } else {
            NN_COUT(stdout, " [FAIL idx=%u]\n", truth + 1);
        }
        fflush(stdout);
        if (!batched) {
            free(in);
            free(out);
        }
    }
    if (hpnn_metrics_active()) {
        char buf[128];
        snprintf(buf, sizeof buf, "\"pass\": %u, \"total\": %u, \"accuracy\": %.6f", g_last_pass, g_last_total,
                 g_last_total ? (double)g_last_pass / g_last_total : 0.0);
        hpnn_metrics_emit("run", buf);
    }
}
