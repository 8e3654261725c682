/*
 * libhpnn caching device allocator (include/libhpnn/devmem.h).
 */
#include <libhpnn.h>
#include <libhpnn/devmem.h>
#include <stdlib.h>

#include <map>
#include <mutex>
#include <unordered_map>
#include <vector>

namespace {

struct Block {
    size_t bytes;
    int dev;
};

std::mutex g_mu;
std::unordered_map<void *, Block> g_live;
std::map<std::pair<int, size_t>, std::vector<void *>> g_free; /* (device, class) -> blocks */
size_t g_in_use = 0, g_cached = 0, g_hits = 0, g_misses = 0;
int g_enabled = -1;

bool enabled() {
    if (g_enabled < 0) {
        const char *e = getenv("HPNN_DEVMEM_CACHE");
        g_enabled = (e && e[0] == '0') ? 0 : 1;
    }
    return g_enabled == 1;
}

/* size classes: 512 B granules up to 1 MiB, then 2 MiB granules */
size_t size_class(size_t n) {
    if (n == 0) n = 1;
    if (n <= (1u << 20)) return (n + 511) / 512 * 512;
    return (n + (2u << 20) - 1) / (2u << 20) * (2u << 20);
}

void release_device(int dev) { /* g_mu held */
    int cur = 0;
    hipGetDevice(&cur);
    for (auto it = g_free.begin(); it != g_free.end();) {
        if (it->first.first != dev) {
            ++it;
            continue;
        }
        hipSetDevice(dev);
        for (void *p : it->second) {
            hipFree(p);
            g_cached -= it->first.second;
        }
        it = g_free.erase(it);
    }
    hipSetDevice(cur);
}

}  // namespace

extern "C" hipError_t hpnn_dev_malloc_raw(void **p, size_t bytes) {
    if (!enabled()) return hipMalloc(p, bytes);
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    const size_t cls = size_class(bytes);
    std::lock_guard<std::mutex> g(g_mu);
    auto it = g_free.find({dev, cls});
    if (it != g_free.end() && !it->second.empty()) {
        *p = it->second.back();
        it->second.pop_back();
        g_cached -= cls;
        g_in_use += cls;
        g_hits++;
        g_live[*p] = {cls, dev};
        return hipSuccess;
    }
    e = hipMalloc(p, cls);
    if (e != hipSuccess) {
        (void)hipGetLastError(); /* clear the sticky OOM, release the cache and retry once */
        release_device(dev);
        e = hipMalloc(p, cls);
        if (e != hipSuccess) return e;
    }
    g_misses++;
    g_in_use += cls;
    g_live[*p] = {cls, dev};
    return hipSuccess;
}

extern "C" hipError_t hpnn_dev_free(void *p) {
    if (!p) return hipSuccess;
    if (!enabled()) return hipFree(p);
    std::lock_guard<std::mutex> g(g_mu);
    auto it = g_live.find(p);
    if (it == g_live.end()) return hipFree(p); /* not ours */
    const Block b = it->second;
    g_live.erase(it);
    /* hipFree semantics: nothing on the owning device may still use the block */
    int cur = 0;
    hipGetDevice(&cur);
    if (cur != b.dev) hipSetDevice(b.dev);
    const hipError_t e = hipDeviceSynchronize();
    if (cur != b.dev) hipSetDevice(cur);
    g_in_use -= b.bytes;
    if (e != hipSuccess) { /* a faulted device: do not recycle */
        hipFree(p);
        return e;
    }
    g_free[{b.dev, b.bytes}].push_back(p);
    g_cached += b.bytes;
    return hipSuccess;
}

extern "C" void hpnn_dev_trim(void) {
    std::lock_guard<std::mutex> g(g_mu);
    std::vector<int> devs;
    for (const auto &kv : g_free) devs.push_back(kv.first.first);
    for (int d : devs) release_device(d);
}

extern "C" void hpnn_dev_stats(size_t *in_use, size_t *cached, size_t *hits, size_t *misses) {
    std::lock_guard<std::mutex> g(g_mu);
    if (in_use) *in_use = g_in_use;
    if (cached) *cached = g_cached;
    if (hits) *hits = g_hits;
    if (misses) *misses = g_misses;
}
