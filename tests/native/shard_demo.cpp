// shard_demo.cpp — the C4 multi-GPU path driven from a native host, without torch: one process per
// GPU, each registering its contiguous block of the jobs against its replica of the map, and the
// 32-B pose records all-gathered over RCCL through the C-ABI (fbr_comm_* / fbr_batch_allgather,
// SURVEY §8(e)).  A ROS / C++ host shards a batch this way.
// Test harness: tests/test_distributed.py writes the input file, runs this program and checks the
// gathered records against its own and the oracle's results.
//
// input : int32 H, W, n_jobs; int64 n_corner_map, n_surf_map; map points (16 B each);
//         per job { float guess[6]; int64 n; n x 24 B fbr_point_xyzirt }
// output: (rank 0) the gathered records of the last launch, rank order, padding removed:
//         n_jobs x {float pose[6]; int32 iterations; int32 status}
// usage : shard_demo IN OUT [--ranks N] [--launches L] [--same-device] [--threads]
//         The parent forks N rank processes before anything touches the GPU; rank 0 writes the
//         RCCL unique id to OUT.id, the others read it (the out-of-band channel a real deployment
//         takes from its launcher).  Rank r uses device r (--same-device: device 0).
//         --threads: one process, one host thread + ctx + rank per device (devices 0..N-1), the
//         communicators made together by fbr_comm_create_local.
// exit  : 0 ok, 2 bad input, 3 library error (prints the status), 4 records differ from the
//         rank's own fbr_batch_results
#include <hip/hip_runtime_api.h>
#include <sys/wait.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "fbr.h"

namespace {
template <class T>
bool rd(FILE* f, T* p, size_t n = 1) {
  return n == 0 || fread(p, sizeof(T), n, f) == n;
}

struct Job {
  float guess[6];
  std::vector<fbr_point_xyzirt> pts;
};

struct Input {
  int32_t H = 0, W = 0, n_jobs = 0;
  std::vector<fbr_point_xyzi> corner, surf;
  std::vector<Job> jobs;
};

bool read_input(const char* path, Input& in) {
  FILE* f = fopen(path, "rb");
  if (!f) return false;
  int64_t nc = 0, ns = 0;
  bool ok = rd(f, &in.H) && rd(f, &in.W) && rd(f, &in.n_jobs) && rd(f, &nc) && rd(f, &ns) && in.n_jobs > 0 &&
            nc >= 0 && ns >= 0;
  if (ok) {
    in.corner.resize(nc);
    in.surf.resize(ns);
    ok = rd(f, in.corner.data(), nc) && rd(f, in.surf.data(), ns);
  }
  for (int j = 0; ok && j < in.n_jobs; ++j) {
    Job jb;
    int64_t n = 0;
    ok = rd(f, jb.guess, 6) && rd(f, &n) && n >= 0;
    if (ok) {
      jb.pts.resize(n);
      ok = rd(f, jb.pts.data(), n);
    }
    in.jobs.push_back(std::move(jb));
  }
  fclose(f);
  return ok;
}

// shard.job_block: rank r owns [total * r / world, total * (r + 1) / world)
int block_begin(int r, int world, int total) { return (int)((int64_t)total * r / world); }

int fail(int rank, const char* what, int st) {
  fprintf(stderr, "rank %d: %s: %s (%d)\n", rank, what, fbr_strerror(st), st);
  return 3;
}

int max_block_of(int world, int n_jobs) {
  int m = 0;
  for (int r = 0; r < world; ++r) m = std::max(m, block_begin(r + 1, world, n_jobs) - block_begin(r, world, n_jobs));
  return m;
}

// One rank's context: created on its device, map set, its block of the jobs staged.
int setup_rank(const Input& in, int rank, int world, int dev, fbr_ctx** out_ctx) {
  *out_ctx = nullptr;
  const int j0 = block_begin(rank, world, in.n_jobs), j1 = block_begin(rank + 1, world, in.n_jobs);
  const int B = j1 - j0;
  fbr_params P;
  fbr_params_default(&P);
  P.n_scan = in.H;
  P.horizon_scan = in.W;
  P.max_batch = std::max(B, 1);
  int64_t nmax = 1;
  for (int j = j0; j < j1; ++j) nmax = std::max<int64_t>(nmax, (int64_t)in.jobs[j].pts.size());
  P.max_points_per_scan = (int32_t)nmax;
  fbr_ctx* ctx = nullptr;
  int st = fbr_create(&ctx, &P, dev);
  if (st) return fail(rank, "fbr_create", st);
  *out_ctx = ctx;
  st = fbr_set_map(ctx, in.corner.data(), (int64_t)in.corner.size(), in.surf.data(), (int64_t)in.surf.size());
  if (st) return fail(rank, "fbr_set_map", st);
  std::vector<const fbr_point_xyzirt*> scans;
  std::vector<int64_t> nin;
  std::vector<float> guesses;
  for (int j = j0; j < j1; ++j) {
    scans.push_back(in.jobs[j].pts.data());
    nin.push_back((int64_t)in.jobs[j].pts.size());
    guesses.insert(guesses.end(), in.jobs[j].guess, in.jobs[j].guess + 6);
  }
  st = fbr_batch_stage(ctx, scans.data(), nin.data(), B, guesses.data());
  if (st) return fail(rank, "fbr_batch_stage", st);
  return 0;
}

// Pipelined launches, each launch's records all-gathered (after launch n, launch n - 1, the same
// launch id on every rank; the last one after the loop), then this rank's own results against its
// block of the gathered records; rank 0 writes the records (rank order, padding removed).
int run_launches(const Input& in, const std::string& out, int rank, int world, int launches, fbr_ctx* ctx,
                 fbr_comm* comm) {
  const int max_block = max_block_of(world, in.n_jobs);
  const int B = block_begin(rank + 1, world, in.n_jobs) - block_begin(rank, world, in.n_jobs);
  void* recv = nullptr;
  const size_t rbytes = sizeof(float) * 8 * (size_t)max_block * world;
  if (hipMalloc(&recv, rbytes) != hipSuccess) return fail(rank, "hipMalloc", FBR_ERR_HIP);
  void* gst = nullptr;
  int st = 0;
  for (int k = 0; k < launches; ++k) {
    st = fbr_batch_launch(ctx);
    if (st) return fail(rank, "fbr_batch_launch", st);
    if (k > 0) {
      st = fbr_batch_allgather(ctx, comm, k - 1, recv, nullptr, &gst);
      if (st) return fail(rank, "fbr_batch_allgather", st);
    }
  }
  st = fbr_batch_allgather(ctx, comm, launches - 1, recv, nullptr, &gst);
  if (st) return fail(rank, "fbr_batch_allgather", st);
  if (hipStreamSynchronize((hipStream_t)gst) != hipSuccess) return fail(rank, "hipStreamSynchronize", FBR_ERR_HIP);
  std::vector<float> rec(8 * (size_t)max_block * world);
  if (hipMemcpy(rec.data(), recv, rbytes, hipMemcpyDeviceToHost) != hipSuccess) return fail(rank, "hipMemcpy", FBR_ERR_HIP);
  std::vector<float> poses(6 * (size_t)B);
  std::vector<fbr_reg_stats> stats(B);
  st = fbr_batch_results(ctx, poses.data(), stats.data());
  if (st) return fail(rank, "fbr_batch_results", st);
  int bad = 0;
  for (int j = 0; j < B; ++j) {
    const float* r = rec.data() + 8 * ((size_t)rank * max_block + j);
    int32_t it, status;
    std::memcpy(&it, r + 6, 4);
    std::memcpy(&status, r + 7, 4);
    bad += std::memcmp(r, poses.data() + 6 * j, 24) != 0 || it != stats[j].iterations || status != stats[j].status;
  }
  if (rank == 0) {
    FILE* f = fopen(out.c_str(), "wb");
    for (int r = 0; f && r < world; ++r) {
      const int n = block_begin(r + 1, world, in.n_jobs) - block_begin(r, world, in.n_jobs);
      fwrite(rec.data() + 8 * (size_t)r * max_block, sizeof(float), 8 * (size_t)n, f);
    }
    if (f) fclose(f);
  }
  (void)hipFree(recv);
  if (bad) {
    fprintf(stderr, "rank %d: %d records differ from fbr_batch_results\n", rank, bad);
    return 4;
  }
  return 0;
}

// Process mode: this process is rank `rank`; the RCCL id travels through OUT.id.
int run_rank(const Input& in, const std::string& out, int rank, int world, int launches, bool same_device) {
  fbr_ctx* ctx = nullptr;
  int rc = setup_rank(in, rank, world, same_device ? 0 : rank, &ctx);
  if (rc) {
    if (ctx) fbr_destroy(ctx);
    return rc;
  }
  // the communicator: rank 0 makes the id, the others take it from OUT.id
  uint8_t id[FBR_COMM_ID_BYTES];
  const std::string idf = out + ".id";
  int st = 0;
  if (rank == 0) {
    st = fbr_comm_unique_id(id);
    if (st) return fail(rank, "fbr_comm_unique_id", st);
    const std::string tmp = idf + ".tmp";
    FILE* f = fopen(tmp.c_str(), "wb");
    if (!f || fwrite(id, 1, sizeof(id), f) != sizeof(id)) return fail(rank, "write id", FBR_ERR_INVALID_ARG);
    fclose(f);
    rename(tmp.c_str(), idf.c_str());
  } else {
    bool got = false;
    for (int t = 0; t < 6000 && !got; ++t) {  // up to 60 s
      FILE* f = fopen(idf.c_str(), "rb");
      if (f) {
        got = fread(id, 1, sizeof(id), f) == sizeof(id);
        fclose(f);
      }
      if (!got) std::this_thread::sleep_for(std::chrono::milliseconds(10));
    }
    if (!got) return fail(rank, "read id", FBR_ERR_STATE);
  }
  fbr_comm* comm = nullptr;
  st = fbr_comm_create(&comm, ctx, id, world, rank, max_block_of(world, in.n_jobs));
  if (st) return fail(rank, "fbr_comm_create", st);
  rc = run_launches(in, out, rank, world, launches, ctx, comm);
  fbr_comm_destroy(comm);
  fbr_destroy(ctx);
  return rc;
}

// Thread mode: one process, one host thread, one ctx and one rank per device.
// The contexts are set up by their threads, the communicators of all of them at once by this
// thread (fbr_comm_create_local: one RCCL group), then every thread runs its launches and gathers.
int run_threads(const Input& in, const std::string& out, int world, int launches) {
  std::vector<fbr_ctx*> ctx(world, nullptr);
  std::vector<int> rc(world, 0);
  {
    std::vector<std::thread> th;
    for (int r = 0; r < world; ++r) th.emplace_back([&, r] { rc[r] = setup_rank(in, r, world, r, &ctx[r]); });
    for (auto& t : th) t.join();
  }
  int first = 0;
  for (int r = 0; r < world; ++r)
    if (rc[r] && !first) first = rc[r];
  std::vector<fbr_comm*> comm(world, nullptr);
  if (!first) {
    const int st = fbr_comm_create_local(comm.data(), ctx.data(), world, max_block_of(world, in.n_jobs));
    if (st) first = fail(0, "fbr_comm_create_local", st);
  }
  if (!first) {
    std::vector<std::thread> th;
    for (int r = 0; r < world; ++r)
      th.emplace_back([&, r] { rc[r] = run_launches(in, out, r, world, launches, ctx[r], comm[r]); });
    for (auto& t : th) t.join();
    for (int r = 0; r < world; ++r)
      if (rc[r] && !first) first = rc[r];
  }
  for (int r = 0; r < world; ++r) {
    if (comm[r]) fbr_comm_destroy(comm[r]);
    if (ctx[r]) fbr_destroy(ctx[r]);
  }
  return first;
}
}  // namespace

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s IN OUT [--ranks N] [--launches L] [--same-device] [--threads]\n", argv[0]);
    return 2;
  }
  int ranks = 1, launches = 3;
  bool same_device = false, threads = false;
  for (int i = 3; i < argc; ++i) {
    if (!strcmp(argv[i], "--ranks") && i + 1 < argc) ranks = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--launches") && i + 1 < argc) launches = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--same-device")) same_device = true;
    else if (!strcmp(argv[i], "--threads")) threads = true;
  }
  Input in;
  if (!read_input(argv[1], in) || ranks < 1 || ranks > in.n_jobs || launches < 1) return 2;
  const std::string out = argv[2];
  if (threads) return run_threads(in, out, ranks, launches);  // rank r on device r
  (void)remove((out + ".id").c_str());
  // one process per rank, forked before any HIP call (the parent never touches the GPU)
  std::vector<pid_t> kids;
  for (int r = 0; r < ranks; ++r) {
    const pid_t p = fork();
    if (p == 0) _exit(run_rank(in, out, r, ranks, launches, same_device));
    if (p < 0) return 3;
    kids.push_back(p);
  }
  int rc = 0;
  for (pid_t p : kids) {
    int ws = 0;
    waitpid(p, &ws, 0);
    const int code = WIFEXITED(ws) ? WEXITSTATUS(ws) : 3;
    if (code && !rc) rc = code;
  }
  return rc;
}
