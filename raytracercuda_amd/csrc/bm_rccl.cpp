// bm_rccl.cpp — RCCL entry points, resolved at first use with dlopen("librccl.so.1").
//
// The library does not link RCCL: single-device contexts never touch it, and in a process where
// torch has already loaded its own RCCL (same soname) dlopen returns that copy, so the process
// holds one RCCL. Only the types come from rccl.h.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <mutex>

#include "bm_internal.h"

namespace bm {

struct Rccl {
    decltype(&ncclGetUniqueId) get_unique_id;
    decltype(&ncclCommInitRank) init_rank;
    decltype(&ncclCommInitAll) init_all;
    decltype(&ncclCommDestroy) destroy;
    decltype(&ncclGroupStart) group_start;
    decltype(&ncclGroupEnd) group_end;
    decltype(&ncclSend) send;
    decltype(&ncclRecv) recv;
    decltype(&ncclGetErrorString) error_string;
};

namespace {
std::once_flag g_once;
Rccl g_rccl;
bool g_ok = false;
const char* g_why = "not loaded";

template <class F>
bool sym(void* h, const char* name, F* out) {
    *out = reinterpret_cast<F>(dlsym(h, name));
    return *out != nullptr;
}

void load_once() {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
        g_why = "librccl.so.1 not found";
        return;
    }
    Rccl r{};
    if (!(sym(h, "ncclGetUniqueId", &r.get_unique_id) && sym(h, "ncclCommInitRank", &r.init_rank) &&
          sym(h, "ncclCommInitAll", &r.init_all) && sym(h, "ncclCommDestroy", &r.destroy) &&
          sym(h, "ncclGroupStart", &r.group_start) && sym(h, "ncclGroupEnd", &r.group_end) &&
          sym(h, "ncclSend", &r.send) && sym(h, "ncclRecv", &r.recv) &&
          sym(h, "ncclGetErrorString", &r.error_string))) {
        g_why = "librccl.so.1 lacks an entry point";
        return;
    }
    g_rccl = r;
    g_ok = true;
    g_why = "";
}
}  // namespace

const Rccl* rccl_load(const char** why) {
    std::call_once(g_once, load_once);
    if (why) *why = g_why;
    return g_ok ? &g_rccl : nullptr;
}

int rccl_unique_id(const Rccl* r, uint8_t* id128) {
    ncclUniqueId id;
    const ncclResult_t e = r->get_unique_id(&id);
    if (e == ncclSuccess) __builtin_memcpy(id128, id.internal, NCCL_UNIQUE_ID_BYTES);
    return (int)e;
}

int rccl_init_rank(const Rccl* r, void** comm, int size, const uint8_t* id128, int rank) {
    ncclUniqueId id;
    __builtin_memcpy(id.internal, id128, NCCL_UNIQUE_ID_BYTES);
    ncclComm_t c = nullptr;
    const ncclResult_t e = r->init_rank(&c, size, id, rank);
    *comm = c;
    return (int)e;
}

int rccl_init_all(const Rccl* r, void** comms, int n, const int* devices) {
    ncclComm_t c[MAX_BAND_SOURCES] = {};
    if (n > (int)MAX_BAND_SOURCES) return (int)ncclInvalidArgument;
    const ncclResult_t e = r->init_all(c, n, devices);
    for (int i = 0; i < n; ++i) comms[i] = c[i];
    return (int)e;
}

void rccl_destroy(const Rccl* r, void* comm) {
    if (comm) (void)r->destroy(reinterpret_cast<ncclComm_t>(comm));
}

int rccl_group_start(const Rccl* r) { return (int)r->group_start(); }
int rccl_group_end(const Rccl* r) { return (int)r->group_end(); }

int rccl_send(const Rccl* r, const void* buf, size_t bytes, int peer, void* comm, hipStream_t s) {
    return (int)r->send(buf, bytes, ncclUint8, peer, reinterpret_cast<ncclComm_t>(comm), s);
}

int rccl_recv(const Rccl* r, void* buf, size_t bytes, int peer, void* comm, hipStream_t s) {
    return (int)r->recv(buf, bytes, ncclUint8, peer, reinterpret_cast<ncclComm_t>(comm), s);
}

const char* rccl_error_string(const Rccl* r, int code) { return r->error_string((ncclResult_t)code); }

}  // namespace bm
