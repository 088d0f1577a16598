// cnf_comm.cpp — the path's one exchange step as C ABI (include/cnf.h): an RCCL communicator per
// process (one process per GPU) and an in-place fp32 sum all-reduce over xGMI.
//
// The reference has no distributed code; the exchange replaces the batch means of
// the log-det (conv_cINN_make_model.py:1323-1326) and of log_loss (:1840-1848) over a batch that
// is sharded across ranks: every rank reduces its own per-image terms (cnf_nll) and one all-reduce
// of the 4 sums (+ the image count) gives the global means.
//
// RCCL is resolved at run time (dlopen of librccl.so.1), so loading libcnf_hip.so never requires it
// and a caller that does not shard never touches it; cnf_comm_init fails with CNF_E_STATE when the
// library is absent.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <cstring>
#include <string>

#include "../../include/cnf.h"

namespace cnf {
int set_error(int code, const char* msg);
}

struct cnf_comm {
    ncclComm_t comm = nullptr;
    int rank = 0, world = 1, device = 0;
};

namespace {

struct Rccl {
    void* h = nullptr;
    ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                               hipStream_t) = nullptr;
    ncclResult_t (*destroy)(ncclComm_t) = nullptr;
    const char* (*err)(ncclResult_t) = nullptr;
    std::string why;
};

const Rccl& rccl() {
    static Rccl r = [] {
        Rccl x;
        for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
            x.h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
            if (x.h) break;
        }
        if (!x.h) {
            const char* e = dlerror();
            x.why = std::string("RCCL not loadable: ") + (e ? e : "librccl.so.1 not found");
            return x;
        }
        x.get_unique_id = reinterpret_cast<decltype(x.get_unique_id)>(dlsym(x.h, "ncclGetUniqueId"));
        x.init_rank = reinterpret_cast<decltype(x.init_rank)>(dlsym(x.h, "ncclCommInitRank"));
        x.all_reduce = reinterpret_cast<decltype(x.all_reduce)>(dlsym(x.h, "ncclAllReduce"));
        x.destroy = reinterpret_cast<decltype(x.destroy)>(dlsym(x.h, "ncclCommDestroy"));
        x.err = reinterpret_cast<decltype(x.err)>(dlsym(x.h, "ncclGetErrorString"));
        if (!x.get_unique_id || !x.init_rank || !x.all_reduce || !x.destroy || !x.err) x.why = "RCCL symbols missing";
        return x;
    }();
    return r;
}

int rccl_fail(const Rccl& r, ncclResult_t e, const char* what) {
    return cnf::set_error(CNF_E_HIP, (std::string(what) + ": " + r.err(e)).c_str());
}

}  // namespace

extern "C" {

int cnf_comm_unique_id(char uid[CNF_COMM_ID_BYTES]) {
    if (!uid) return cnf::set_error(CNF_E_INVALID, "null uid");
    const Rccl& r = rccl();
    if (!r.why.empty()) return cnf::set_error(CNF_E_STATE, r.why.c_str());
    ncclUniqueId id;
    ncclResult_t e = r.get_unique_id(&id);
    if (e != ncclSuccess) return rccl_fail(r, e, "ncclGetUniqueId");
    static_assert(sizeof(id.internal) == CNF_COMM_ID_BYTES, "unique id size");
    std::memcpy(uid, id.internal, CNF_COMM_ID_BYTES);
    return CNF_OK;
}

int cnf_comm_init(int rank, int world, const char uid[CNF_COMM_ID_BYTES], cnf_comm** out) {
    if (!out || !uid) return cnf::set_error(CNF_E_INVALID, "null argument");
    *out = nullptr;
    if (world < 1 || rank < 0 || rank >= world) return cnf::set_error(CNF_E_INVALID, "rank / world out of range");
    const Rccl& r = rccl();
    if (!r.why.empty()) return cnf::set_error(CNF_E_STATE, r.why.c_str());
    cnf_comm* c = new cnf_comm;
    c->rank = rank;
    c->world = world;
    if (hipGetDevice(&c->device) != hipSuccess) {
        delete c;
        return cnf::set_error(CNF_E_HIP, "hipGetDevice");
    }
    ncclUniqueId id;
    std::memcpy(id.internal, uid, CNF_COMM_ID_BYTES);
    ncclResult_t e = r.init_rank(&c->comm, world, id, rank);
    if (e != ncclSuccess) {
        delete c;
        return rccl_fail(r, e, "ncclCommInitRank");
    }
    *out = c;
    return CNF_OK;
}

int cnf_allreduce_sum_f32(cnf_comm* comm, float* buf, size_t n, void* stream) {
    if (!comm || (!buf && n)) return cnf::set_error(CNF_E_INVALID, "null argument");
    if (n == 0) return CNF_OK;
    const Rccl& r = rccl();
    ncclResult_t e = r.all_reduce(buf, buf, n, ncclFloat32, ncclSum, comm->comm, (hipStream_t)stream);
    if (e != ncclSuccess) return rccl_fail(r, e, "ncclAllReduce");
    return CNF_OK;
}

int cnf_nll_allreduce(cnf_comm* comm, const float* sums, int B, float* red5, void* stream) {
    if (!sums || !red5 || B < 0) return cnf::set_error(CNF_E_INVALID, "null argument or B < 0");
    const hipStream_t st = (hipStream_t)stream;
    // pack (sums[0..3], B) with two stream-ordered copies (capturable, no kernel), then one all-reduce
    if (hipMemcpyAsync(red5, sums, 4 * sizeof(float), hipMemcpyDeviceToDevice, st) != hipSuccess)
        return cnf::set_error(CNF_E_HIP, "hipMemcpyAsync(sums)");
    const float fb = (float)B;
    uint32_t bits;
    std::memcpy(&bits, &fb, 4);
    if (hipMemsetD32Async((hipDeviceptr_t)(red5 + 4), (int)bits, 1, st) != hipSuccess)
        return cnf::set_error(CNF_E_HIP, "hipMemsetD32Async(B)");
    if (!comm) return CNF_OK;
    return cnf_allreduce_sum_f32(comm, red5, 5, stream);
}

void cnf_comm_destroy(cnf_comm* comm) {
    if (!comm) return;
    if (comm->comm) (void)rccl().destroy(comm->comm);
    delete comm;
}

}  // extern "C"
