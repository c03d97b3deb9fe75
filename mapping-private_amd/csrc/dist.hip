// dist.hip -- the multi-GPU exchange of the frame-sharded path.
//
// Frames are independent: each process drives one GPU and takes its own shard of frames,
// with no data-path collective.  The one exchange is the gather of every rank's
// detection records after a batch (M x rank c3h_det per frame, 24 B each): one RCCL
// all-gather on the context's stream over xGMI, latency-bound at these sizes.  The caller
// owns the communicator (ncclCommInitRank with its own id exchange, as torch.distributed
// does); librccl is loaded at the first call, so single-GPU users never load it.
#include <dlfcn.h>

#include <mutex>
#include <string>

#include <rccl/rccl.h>  // types and prototypes only

#include "c3h_internal.h"

namespace {

struct Rccl {
  std::once_flag once;
  bool ok = false;
  std::string err;
  decltype(&ncclAllGather) allgather = nullptr;
  decltype(&ncclGetErrorString) errstr = nullptr;
};
Rccl g_rccl;

bool rccl_load() {
  std::call_once(g_rccl.once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
      g_rccl.err = std::string("cannot load RCCL: ") + dlerror();
      return;
    }
    g_rccl.allgather = (decltype(g_rccl.allgather))dlsym(h, "ncclAllGather");
    g_rccl.errstr = (decltype(g_rccl.errstr))dlsym(h, "ncclGetErrorString");
    g_rccl.ok = g_rccl.allgather != nullptr;
    if (!g_rccl.ok) g_rccl.err = "RCCL symbols missing";
  });
  return g_rccl.ok;
}

}  // namespace

extern "C" int c3h_allgather_detections(c3h_ctx* ctx, void* nccl_comm, const c3h_det* d_local, int64_t n_local,
                                        c3h_det* d_all) {
  if (!ctx || !nccl_comm || n_local < 0 || (n_local > 0 && (!d_local || !d_all))) return C3H_ERR_ARG;
  int rc = c3h_stream_flush(ctx);  // an open frame stream's last batches first (stream order)
  if (rc != C3H_OK) return rc;
  if (n_local == 0) return C3H_OK;
  if (!rccl_load()) {
    ctx->err = g_rccl.err;
    return C3H_ERR_HIP;
  }
  if (hipSetDevice(ctx->device) != hipSuccess) return C3H_ERR_HIP;
  const ncclResult_t r = g_rccl.allgather(d_local, d_all, (size_t)n_local * sizeof(c3h_det), ncclUint8,
                                          (ncclComm_t)nccl_comm, ctx->stream);
  if (r != ncclSuccess) {
    ctx->err = std::string("ncclAllGather: ") + (g_rccl.errstr ? g_rccl.errstr(r) : "error");
    return C3H_ERR_HIP;
  }
  return C3H_OK;
}
