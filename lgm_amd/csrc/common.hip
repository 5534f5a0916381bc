// lgm_amd/csrc/common.hip -- error string + the per-call HIP-event profiler (include/lgm_common.h).
#include "common.h"

#include <stdarg.h>
#include <string.h>

#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "lgm_common.h"

struct lgm_profiler {
    struct Rec { const char *name; hipEvent_t a, b; };
    std::mutex mu;
    std::vector<Rec> recs;
    std::vector<hipEvent_t> pool;
    size_t used = 0;
    hipEvent_t get() {
        if (used == pool.size()) {
            hipEvent_t e;
            if (hipEventCreate(&e) != hipSuccess) return nullptr;
            pool.push_back(e);
        }
        return pool[used++];
    }
};

namespace lgm {
static thread_local char g_err[512] = {0};
static thread_local const lgm_diag *g_call_diag = nullptr;  // only while an entry point runs (DiagScope)
static thread_local const char *g_pending = nullptr;
static thread_local hipEvent_t g_pending_ev = nullptr;

void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}
void clear_error() { g_err[0] = 0; }

static thread_local int g_scope_depth = 0;
DiagScope::DiagScope(const lgm_diag *d) {
    if (g_scope_depth++ == 0) g_call_diag = d;  // (an entry point called from another keeps the outer call's)
}
DiagScope::~DiagScope() {
    if (--g_scope_depth == 0) {
        g_call_diag = nullptr;
        g_pending_ev = nullptr;
    }
}
const lgm_diag *call_diag() { return g_call_diag; }

static lgm_profiler *call_profiler() { return g_call_diag ? g_call_diag->profiler : nullptr; }

void prof_begin(const char *name, hipStream_t st) {
    lgm_profiler *p = call_profiler();
    if (!p) return;
    std::lock_guard<std::mutex> lk(p->mu);
    g_pending = name;
    g_pending_ev = p->get();
    if (g_pending_ev) (void)hipEventRecord(g_pending_ev, st);
}
void prof_end(hipStream_t st) {
    lgm_profiler *p = call_profiler();
    if (!p || !g_pending_ev) return;
    std::lock_guard<std::mutex> lk(p->mu);
    hipEvent_t b = p->get();
    if (!b) return;
    (void)hipEventRecord(b, st);
    p->recs.push_back({g_pending, g_pending_ev, b});
    g_pending_ev = nullptr;
}
}  // namespace lgm

extern "C" {
const char *lgm_last_error(void) { return lgm::g_err; }
int lgm_abi_version(void) { return 5; }

lgm_profiler *lgm_profiler_create(void) { return new lgm_profiler(); }
int lgm_profiler_reset(lgm_profiler *p) {
    if (!p) return LGM_E_INVALID;
    std::lock_guard<std::mutex> lk(p->mu);
    p->recs.clear();
    p->used = 0;
    return LGM_OK;
}
int lgm_profiler_summary(lgm_profiler *p, char *buf, size_t len) {
    if (!p || !buf || len == 0) return LGM_E_INVALID;
    std::map<std::string, std::pair<int, double>> agg;
    std::vector<std::string> order;
    for (auto &r : p->recs) {
        if (hipEventSynchronize(r.b) != hipSuccess) {
            lgm::set_error("event sync failed");
            return LGM_E_HIP;
        }
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, r.a, r.b);
        auto it = agg.find(r.name);
        if (it == agg.end()) {
            order.push_back(r.name);
            agg[r.name] = {1, ms};
        } else {
            it->second.first++;
            it->second.second += ms;
        }
    }
    std::string out;
    char line[256];
    for (auto &n : order) {
        snprintf(line, sizeof(line), "%s %d %.6f\n", n.c_str(), agg[n].first, agg[n].second);
        out += line;
    }
    strncpy(buf, out.c_str(), len - 1);
    buf[len - 1] = 0;
    return LGM_OK;
}
void lgm_profiler_destroy(lgm_profiler *p) {
    if (!p) return;
    for (auto e : p->pool) (void)hipEventDestroy(e);
    delete p;
}
}
