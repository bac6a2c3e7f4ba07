// rccl_loopback.cpp -- TEST TRANSPORT ONLY: the subset of the RCCL C API that
// sfrt_multi.cpp calls, implemented with HIP peer copies, so that sfrt_multi's RCCL
// branch (ncclCommInitAll, in-place ncclGather, grouped ncclSend/ncclRecv, packed
// send -> unpack) runs with n > 1 ranks on a one-GPU box.  Real RCCL refuses a device
// listed twice in ncclCommInitAll; this library accepts it.  Loaded by libsfrt.so in
// place of librccl.so.1 after an explicit sfrt_multi_use_test_transport(path) call made
// before the process's first RCCL context (tests/test_gpu_bands.py).
//
// Ordering contract (RCCL's, for what sfrt_multi relies on): an operation queued on a
// rank's stream starts after the work queued on that stream before it, and every
// participating rank's stream waits until the operation's data movement is done.
// Inside ncclGroupStart/End the operations are matched at ncclGroupEnd: a gather
// once all ranks of the communicator posted theirs; a send with the receive its
// receiver posted for it (FIFO per sender/receiver pair).  Each transfer is a
// hipMemcpyPeerAsync on the receiver's stream after an event of the sender's stream,
// and the sender's stream then waits for an event after the copy.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <cstdint>
#include <deque>
#include <map>
#include <mutex>
#include <utility>
#include <vector>

struct Clique;

struct ncclComm {
  Clique* clique;
  int rank;
  int device;
};

namespace {

struct Post {
  ncclComm* comm;
  const void* send;
  void* recv;
  size_t bytes;
  int peer;  // gather: root; send: receiver; recv: sender
  hipStream_t stream;
};

std::mutex mu;
int group_depth = 0;
std::vector<Post> pending_gathers;
std::map<std::pair<Clique*, std::pair<int, int>>, std::deque<Post>> sends, recvs;  // (src, dst)

// stats for the tests (rccl_loopback_stats)
std::atomic<long long> n_gather{0}, n_send{0}, n_recv{0}, n_copies{0}, bytes_copied{0};

size_t type_size(ncclDataType_t t) {
  switch (t) {
    case ncclInt8: case ncclUint8: case ncclFloat8e4m3: case ncclFloat8e5m2: return 1;
    case ncclFloat16: case ncclBfloat16: return 2;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    default: return 8;
  }
}

struct Guard {
  int old = 0;
  explicit Guard(int d) {
    (void)hipGetDevice(&old);
    (void)hipSetDevice(d);
  }
  ~Guard() { (void)hipSetDevice(old); }
};

// src (on src_dev, queued on s_src) -> dst (on dst_dev, queued on s_dst).
ncclResult_t transfer(void* dst, int dst_dev, hipStream_t s_dst, const void* src, int src_dev,
                      hipStream_t s_src, size_t bytes) {
  hipEvent_t sent, done;
  {
    Guard g(src_dev);
    if (hipEventCreateWithFlags(&sent, hipEventDisableTiming) != hipSuccess ||
        hipEventRecord(sent, s_src) != hipSuccess)
      return ncclUnhandledCudaError;
  }
  {
    Guard g(dst_dev);
    if (hipEventCreateWithFlags(&done, hipEventDisableTiming) != hipSuccess ||
        hipStreamWaitEvent(s_dst, sent, 0) != hipSuccess)
      return ncclUnhandledCudaError;
    if (bytes && dst != src &&
        hipMemcpyPeerAsync(dst, dst_dev, src, src_dev, bytes, s_dst) != hipSuccess)
      return ncclUnhandledCudaError;
    if (hipEventRecord(done, s_dst) != hipSuccess) return ncclUnhandledCudaError;
  }
  {
    Guard g(src_dev);
    if (hipStreamWaitEvent(s_src, done, 0) != hipSuccess) return ncclUnhandledCudaError;
  }
  (void)hipEventDestroy(sent);
  (void)hipEventDestroy(done);
  n_copies++;
  bytes_copied += (long long)bytes;
  return ncclSuccess;
}

}  // namespace

struct Clique {
  int n;
};

namespace {

// Match and run everything posted (called at the outermost ncclGroupEnd, or right away
// outside a group).  Returns ncclInvalidUsage for posts left unmatched at a group end.
ncclResult_t flush(bool group_end) {
  ncclResult_t rc = ncclSuccess;
  // gathers: per (clique, root) once every rank posted
  std::map<std::pair<Clique*, int>, std::vector<Post>> by_root;
  for (const Post& p : pending_gathers) by_root[{p.comm->clique, p.peer}].push_back(p);
  std::vector<Post> left;
  for (auto& kv : by_root) {
    auto& v = kv.second;
    Clique* c = kv.first.first;
    if ((int)v.size() < c->n) {
      left.insert(left.end(), v.begin(), v.end());
      continue;
    }
    const Post* root = nullptr;
    for (const Post& p : v)
      if (p.comm->rank == kv.first.second) root = &p;
    if (!root) return ncclInvalidUsage;
    for (const Post& p : v) {
      void* dst = (uint8_t*)root->recv + (size_t)p.comm->rank * p.bytes;
      if ((rc = transfer(dst, root->comm->device, root->stream, p.send, p.comm->device, p.stream,
                         p.bytes)) != ncclSuccess)
        return rc;
    }
  }
  pending_gathers.swap(left);
  // point to point: FIFO per (sender, receiver)
  for (auto& kv : sends) {
    auto it = recvs.find(kv.first);
    if (it == recvs.end()) continue;
    auto& sq = kv.second;
    auto& rq = it->second;
    while (!sq.empty() && !rq.empty()) {
      const Post s = sq.front(), r = rq.front();
      sq.pop_front();
      rq.pop_front();
      if (s.bytes != r.bytes) return ncclInvalidUsage;
      if ((rc = transfer(r.recv, r.comm->device, r.stream, s.send, s.comm->device, s.stream,
                         s.bytes)) != ncclSuccess)
        return rc;
    }
  }
  if (group_end) {
    bool unmatched = !pending_gathers.empty();
    for (auto& kv : sends) unmatched = unmatched || !kv.second.empty();
    for (auto& kv : recvs) unmatched = unmatched || !kv.second.empty();
    if (unmatched) {
      pending_gathers.clear();
      sends.clear();
      recvs.clear();
      return ncclInvalidUsage;  // RCCL would hang; a test transport fails loudly instead
    }
  }
  return ncclSuccess;
}

}  // namespace

extern "C" {

ncclResult_t ncclCommInitAll(ncclComm_t* comm, int ndev, const int* devlist) {
  if (!comm || ndev <= 0) return ncclInvalidArgument;
  Clique* c = new Clique{ndev};
  for (int r = 0; r < ndev; r++) comm[r] = new ncclComm{c, r, devlist ? devlist[r] : r};
  return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
  if (!comm) return ncclInvalidArgument;
  delete comm;  // the clique is shared by the communicators (leaked: test library)
  return ncclSuccess;
}

ncclResult_t ncclGroupStart() {
  std::lock_guard<std::mutex> lk(mu);
  group_depth++;
  return ncclSuccess;
}

ncclResult_t ncclGroupEnd() {
  std::lock_guard<std::mutex> lk(mu);
  if (group_depth <= 0) return ncclInvalidUsage;
  if (--group_depth > 0) return ncclSuccess;
  return flush(true);
}

ncclResult_t ncclGather(const void* sendbuff, void* recvbuff, size_t sendcount,
                        ncclDataType_t datatype, int root, ncclComm_t comm, hipStream_t stream) {
  if (!comm || root < 0 || root >= comm->clique->n) return ncclInvalidArgument;
  std::lock_guard<std::mutex> lk(mu);
  n_gather++;
  pending_gathers.push_back(
      Post{comm, sendbuff, recvbuff, sendcount * type_size(datatype), root, stream});
  return group_depth ? ncclSuccess : flush(false);
}

ncclResult_t ncclSend(const void* sendbuff, size_t count, ncclDataType_t datatype, int peer,
                      ncclComm_t comm, hipStream_t stream) {
  if (!comm || peer < 0 || peer >= comm->clique->n) return ncclInvalidArgument;
  std::lock_guard<std::mutex> lk(mu);
  n_send++;
  sends[{comm->clique, {comm->rank, peer}}].push_back(
      Post{comm, sendbuff, nullptr, count * type_size(datatype), peer, stream});
  return group_depth ? ncclSuccess : flush(false);
}

ncclResult_t ncclRecv(void* recvbuff, size_t count, ncclDataType_t datatype, int peer,
                      ncclComm_t comm, hipStream_t stream) {
  if (!comm || peer < 0 || peer >= comm->clique->n) return ncclInvalidArgument;
  std::lock_guard<std::mutex> lk(mu);
  n_recv++;
  recvs[{comm->clique, {peer, comm->rank}}].push_back(
      Post{comm, nullptr, recvbuff, count * type_size(datatype), peer, stream});
  return group_depth ? ncclSuccess : flush(false);
}

// gathers, sends, receives posted; peer copies issued; bytes copied
void rccl_loopback_stats(long long* out5) {
  out5[0] = n_gather;
  out5[1] = n_send;
  out5[2] = n_recv;
  out5[3] = n_copies;
  out5[4] = bytes_copied;
}

}  // extern "C"
