/*
 * libhpnn observability layer (include/libhpnn/observe.h): trace ranges forwarded to
 * roctx + a host-side timing table, JSON-lines metrics, debug mode.
 *
 * The reference has no timing or trace code at all; its only debug aids
 * are CHK_ERR after launches in DEBUG builds (common.h:324-335) and the DBG_TRACE /
 * CUDA_TRACE_V array sums (ann.h:29-33, common.h:486-490).
 */
#include <libhpnn/observe.h>
#include <dlfcn.h>
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <map>
#include <mutex>
#include <string>
#include <vector>

namespace {

struct Roctx {
    int (*push)(const char *) = nullptr;
    int (*pop)() = nullptr;
    bool tried = false;
    void load() {
        if (tried) return;
        tried = true;
        const char *names[] = {"libroctx64.so.4", "libroctx64.so", "/opt/rocm/lib/libroctx64.so.4"};
        for (const char *n : names) {
            void *h = dlopen(n, RTLD_NOW | RTLD_LOCAL);
            if (!h) continue;
            push = (int (*)(const char *))dlsym(h, "roctxRangePushA");
            pop = (int (*)())dlsym(h, "roctxRangePop");
            if (push && pop) return;
            push = nullptr;
            pop = nullptr;
        }
    }
};

struct Entry {
    UINT64 calls = 0;
    double seconds = 0.0;
};

struct Frame {
    std::string name;
    std::chrono::steady_clock::time_point t0;
};

std::mutex g_mu;
int g_trace = -1; /* -1: not read from the environment yet */
Roctx g_roctx;
std::map<std::string, Entry> g_table;
thread_local std::vector<Frame> t_stack;

FILE *g_metrics = nullptr;
bool g_metrics_env_read = false;
int g_debug = -1;

int trace_on() {
    if (g_trace < 0) {
        const char *e = getenv("HPNN_TRACE");
        g_trace = (e && e[0] && e[0] != '0') ? 1 : 0;
    }
    return g_trace;
}

}  // namespace

extern "C" int hpnn_trace_enabled(void) { return trace_on(); }

extern "C" void hpnn_trace_enable(int on) {
    std::lock_guard<std::mutex> g(g_mu);
    g_trace = on ? 1 : 0;
}

extern "C" void hpnn_trace_push(const char *name) {
    if (!trace_on()) return;
    {
        std::lock_guard<std::mutex> g(g_mu);
        g_roctx.load();
    }
    if (g_roctx.push) g_roctx.push(name);
    t_stack.push_back({name, std::chrono::steady_clock::now()});
}

extern "C" void hpnn_trace_pop(void) {
    if (t_stack.empty()) return;
    const Frame f = t_stack.back();
    t_stack.pop_back();
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - f.t0).count();
    if (g_roctx.pop) g_roctx.pop();
    hpnn_trace_add(f.name.c_str(), s);
}

extern "C" void hpnn_trace_add(const char *name, double seconds) {
    std::lock_guard<std::mutex> g(g_mu);
    Entry &e = g_table[name];
    e.calls++;
    e.seconds += seconds;
}

extern "C" int hpnn_trace_report(FILE *fp) {
    std::lock_guard<std::mutex> g(g_mu);
    if (g_table.empty() || hpnn_output_rank() != 0) return (int)g_table.size();
    fprintf(fp, "NN(TRACE): %-32s %10s %12s %12s\n", "range", "calls", "total ms", "mean us");
    for (const auto &kv : g_table)
        fprintf(fp, "NN(TRACE): %-32s %10llu %12.3f %12.3f\n", kv.first.c_str(), (unsigned long long)kv.second.calls,
                kv.second.seconds * 1e3, kv.second.calls ? kv.second.seconds * 1e6 / kv.second.calls : 0.0);
    fflush(fp);
    return (int)g_table.size();
}

extern "C" void hpnn_trace_reset(void) {
    std::lock_guard<std::mutex> g(g_mu);
    g_table.clear();
}

extern "C" UINT64 hpnn_trace_calls(const char *name) {
    std::lock_guard<std::mutex> g(g_mu);
    auto it = g_table.find(name);
    return it == g_table.end() ? 0 : it->second.calls;
}

extern "C" double hpnn_trace_seconds(const char *name) {
    std::lock_guard<std::mutex> g(g_mu);
    auto it = g_table.find(name);
    return it == g_table.end() ? 0.0 : it->second.seconds;
}

/* ---------------------------------------------------------------- metrics */
extern "C" int hpnn_metrics_open(const char *path) {
    std::lock_guard<std::mutex> g(g_mu);
    g_metrics_env_read = true;
    if (g_metrics) {
        fclose(g_metrics);
        g_metrics = nullptr;
    }
    if (!path || !path[0]) return 0;
    if (hpnn_output_rank() != 0) return 0; /* rank 0 writes the record stream */
    g_metrics = fopen(path, "a");
    if (!g_metrics) {
        NN_ERROR(stderr, "can't open metrics file %s\n", path);
        return -1;
    }
    return 0;
}

extern "C" int hpnn_metrics_active(void) {
    if (!g_metrics_env_read) {
        const char *e = getenv("HPNN_METRICS");
        if (e && e[0]) hpnn_metrics_open(e);
        g_metrics_env_read = true;
    }
    return g_metrics != nullptr;
}

extern "C" void hpnn_metrics_emit(const char *event, const char *fields) {
    if (!hpnn_metrics_active()) return;
    std::lock_guard<std::mutex> g(g_mu);
    if (!g_metrics) return;
    const double t = std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count();
    fprintf(g_metrics, "{\"event\": \"%s\", \"time\": %.6f%s%s}\n", event, t, (fields && fields[0]) ? ", " : "",
            fields ? fields : "");
    fflush(g_metrics);
}

extern "C" void hpnn_metrics_epoch(const char *engine, UINT epoch, double loss, UINT correct, UINT n, double seconds,
                                   UINT64 samples) {
    if (!hpnn_metrics_active()) return;
    char buf[512];
    snprintf(buf, sizeof buf,
             "\"engine\": \"%s\", \"epoch\": %u, \"loss\": %.10g, \"correct\": %u, \"n\": %u, \"accuracy\": %.6f, "
             "\"seconds\": %.6f, \"samples\": %llu, \"samples_per_s\": %.3f",
             engine, epoch, loss, correct, n, n ? (double)correct / n : 0.0, seconds, (unsigned long long)samples,
             seconds > 0 ? samples / seconds : 0.0);
    hpnn_metrics_emit("epoch", buf);
}

/* ---------------------------------------------------------------- debug */
extern "C" int hpnn_debug_enabled(void) {
    if (g_debug < 0) {
        const char *e = getenv("HPNN_DEBUG");
        g_debug = (e && e[0] && e[0] != '0') ? 1 : 0;
    }
    return g_debug;
}

extern "C" int hpnn_debug_check(const char *where) {
    if (!hpnn_debug_enabled()) return 0;
    hipError_t e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipGetLastError();
    if (e != hipSuccess) {
        NN_ERROR(stderr, "HIP error after %s: %s\n", where, hipGetErrorString(e));
        return -1;
    }
    return 0;
}
