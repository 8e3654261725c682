/*
 * libhpnn observability: tracing ranges, phase timers, structured metrics, debug mode.
 *
 * The reference has no timers, no trace hooks and only verbosity-gated log lines
 * ("Tracing / profiling: None", "Metrics / logging").  This layer adds:
 *
 *   - trace ranges (HPNN_TRACE=1): hpnn_trace_push/pop nest named ranges that are
 *     forwarded to roctx (libroctx64, dlopen'ed on first use, so `rocprofv3
 *     --marker-trace` shows them on the timeline) and accumulated in a host-side
 *     table of {calls, total seconds} per name; hpnn_trace_report prints the table
 *     (train_nn does at exit when tracing is on).
 *   - metrics (HPNN_METRICS=<file>): JSON-lines records appended by the training
 *     drivers, one per epoch (batched) or one per sample (online), plus a summary
 *     record; rank 0 only under a launcher.
 *   - debug mode (HPNN_DEBUG=1, read by nn_init_all before the HIP runtime starts):
 *     AMD_SERIALIZE_KERNEL=3 / AMD_SERIALIZE_COPY=3 (every launch and copy is
 *     synchronous and checked, so a faulting kernel is reported at its launch) and
 *     hpnn_debug_check() after every engine launch sequence.
 */
#ifndef LIBHPNN_OBSERVE_H
#define LIBHPNN_OBSERVE_H
#include <libhpnn.h>

#ifdef __cplusplus
extern "C" {
#endif

/* tracing */
int hpnn_trace_enabled(void);
void hpnn_trace_enable(int on);
void hpnn_trace_push(const char *name);
void hpnn_trace_pop(void);
/* adds `seconds` to the table entry `name` (device-side phase times measured with
 * hipEvents by the engines) */
void hpnn_trace_add(const char *name, double seconds);
/* prints the table (name, calls, total ms, mean us) to fp; returns #entries */
int hpnn_trace_report(FILE *fp);
void hpnn_trace_reset(void);
/* number of calls / total seconds recorded for name (0 if absent) */
UINT64 hpnn_trace_calls(const char *name);
double hpnn_trace_seconds(const char *name);

/* metrics: open the JSON-lines sink (NULL closes it); HPNN_METRICS opens it lazily */
int hpnn_metrics_open(const char *path);
int hpnn_metrics_active(void);
/* appends {"event": event, <fields>} where fields is a JSON object body without braces,
 * e.g. "\"epoch\": 1, \"loss\": 0.25" */
void hpnn_metrics_emit(const char *event, const char *fields);
/* epoch record of the batched drivers */
void hpnn_metrics_epoch(const char *engine, UINT epoch, double loss, UINT correct, UINT n, double seconds,
                        UINT64 samples);

/* debug mode */
int hpnn_debug_enabled(void);
/* HPNN_DEBUG: synchronise the current device and report any pending HIP error with the
 * call site; returns 0 when healthy (always 0 outside debug mode) */
int hpnn_debug_check(const char *where);

/* RAII range for C++ callers */
#ifdef __cplusplus
}
struct HpnnTraceRange {
    explicit HpnnTraceRange(const char *n) : on(hpnn_trace_enabled()) {
        if (on) hpnn_trace_push(n);
    }
    ~HpnnTraceRange() {
        if (on) hpnn_trace_pop();
    }
    int on;
};
#endif
#endif
