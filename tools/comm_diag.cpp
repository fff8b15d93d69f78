// comm_diag.cpp — where RCCL's communicator setup blocks when a peer never
// joins (VERDICT r03 "next" 1: find the cause of the init/abort hang from
// evidence, in ONE run per mode, not by repetition).
//
// One process, one GPU. Rank 0 of a 2-rank communicator is initialised with
// a fresh unique id (the bootstrap root thread lives in this process, created
// by ncclGetUniqueId) and rank 1 never arrives. A watcher thread snapshots
// every thread of the process from /proc/self/task (name, state, wchan,
// current syscall) at fixed times, so the blocking call and the thread it
// waits on are named by the kernel's own view.
//
//   mode "nb"   ncclCommInitRankConfig(blocking = 0) on the calling thread:
//               how long the call itself takes to return, then the async
//               state for 3 s, then ncclCommAbort (bounded observation 20 s)
//   mode "nb2"  the same as the process's second communicator (a 1-rank
//               communicator is created and destroyed first)
//   mode "blk"  the blocking form on a helper thread, then ncclCommAbort
//
//   hipcc -O2 -std=c++17 tools/comm_diag.cpp -o tools/comm_diag -lrccl -lpthread
//   NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=INIT,BOOTSTRAP tools/comm_diag nb
#include <dirent.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>

static double t0;
static double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static std::string slurp(const std::string& p) {
  FILE* f = fopen(p.c_str(), "r");
  if (!f) return "?";
  char b[512];
  size_t n = fread(b, 1, sizeof b - 1, f);
  fclose(f);
  b[n] = 0;
  std::string s(b);
  while (!s.empty() && (s.back() == '\n' || s.back() == ' ')) s.pop_back();
  return s;
}

static const char* sysname(long nr) {
  switch (nr) {
    case 0: return "read";
    case 7: return "poll";
    case 23: return "select";
    case 35: return "nanosleep";
    case 42: return "connect";
    case 43: return "accept";
    case 45: return "recvfrom";
    case 47: return "recvmsg";
    case 202: return "futex";
    case 230: return "clock_nanosleep";
    case 232: return "epoll_wait";
    case 270: return "pselect6";
    case 271: return "ppoll";
    case 281: return "epoll_pwait";
    case 288: return "accept4";
    case 16: return "ioctl";
    default: return "";
  }
}

// one line per thread: tid name state wchan syscall
static void snapshot(const char* tag) {
  printf("--- snapshot %s at %.3f s\n", tag, now_s() - t0);
  DIR* d = opendir("/proc/self/task");
  if (!d) return;
  while (dirent* e = readdir(d)) {
    if (e->d_name[0] == '.') continue;
    const std::string base = std::string("/proc/self/task/") + e->d_name;
    const std::string stat = slurp(base + "/stat");
    char state = '?';
    const size_t rp = stat.rfind(')');
    if (rp != std::string::npos && rp + 2 < stat.size()) state = stat[rp + 2];
    const std::string sc = slurp(base + "/syscall");
    long nr = -1;
    if (!sc.empty() && sc[0] != 'r' && sc[0] != '?') nr = strtol(sc.c_str(), nullptr, 10);
    printf("  tid %-7s %-16s %c wchan=%-24s syscall=%ld %s\n", e->d_name, slurp(base + "/comm").c_str(),
           state, slurp(base + "/wchan").c_str(), nr, nr >= 0 ? sysname(nr) : sc.c_str());
  }
  closedir(d);
  fflush(stdout);
}

static int nthreads() {
  int n = 0;
  DIR* d = opendir("/proc/self/task");
  while (dirent* e = readdir(d)) n += e->d_name[0] != '.';
  closedir(d);
  return n;
}

int main(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "nb";
  t0 = now_s();
  setvbuf(stdout, nullptr, _IOLBF, 0);
  if (hipSetDevice(0) != hipSuccess) return 3;
  (void)hipFree(nullptr);
  printf("mode %s, threads at start %d\n", mode.c_str(), nthreads());
  if (mode == "nb2") {  // a first, successful communicator
    ncclComm_t c1;
    ncclUniqueId id1;
    ncclGetUniqueId(&id1);
    const ncclResult_t r = ncclCommInitRank(&c1, 1, id1, 0);
    printf("1-rank communicator: %d at %.3f s\n", (int)r, now_s() - t0);
    ncclCommDestroy(c1);
    printf("threads after the 1-rank communicator %d\n", nthreads());
  }
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  printf("ncclGetUniqueId: %d at %.3f s; threads %d\n", (int)r, now_s() - t0, nthreads());
  snapshot("after unique id");
  ncclComm_t comm = nullptr;
  std::atomic<bool> returned{false};
  std::thread helper;
  if (mode == "blk") {
    helper = std::thread([&] {
      ncclComm_t c = nullptr;
      const ncclResult_t rr = ncclCommInitRank(&c, 2, id, 0);
      printf("blocking init returned %d at %.3f s\n", (int)rr, now_s() - t0);
      returned = true;
    });
  } else {
    // the non-blocking call on this thread, watched from a second one
    std::atomic<bool> stop{false};
    std::thread watch([&] {
      for (int k = 0; k < 40 && !stop; k++) {
        std::this_thread::sleep_for(std::chrono::milliseconds(500));
        if (!stop) snapshot("while ncclCommInitRankConfig has not returned");
      }
    });
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    const double a = now_s();
    r = ncclCommInitRankConfig(&comm, 2, id, 0, &cfg);
    stop = true;
    watch.join();
    printf("ncclCommInitRankConfig(blocking=0) returned %d (%s) after %.3f s; threads %d\n", (int)r,
           ncclGetErrorString(r), now_s() - a, nthreads());
  }
  for (int k = 0; k < 6; k++) {
    std::this_thread::sleep_for(std::chrono::milliseconds(500));
    if (comm) {
      ncclResult_t st = ncclSuccess;
      ncclCommGetAsyncError(comm, &st);
      printf("async state %d at %.3f s\n", (int)st, now_s() - t0);
    }
  }
  snapshot("3 s after the init call");
  if (!comm) {
    printf("no communicator handle to abort (blocking form still inside the call: %s)\n",
           returned ? "no" : "yes");
    fflush(stdout);
    _exit(0);  // the helper is stuck inside RCCL; nothing else to observe
  }
  std::atomic<bool> aborted{false};
  std::thread ab([&] {
    const double a = now_s();
    const ncclResult_t ra = ncclCommAbort(comm);
    printf("ncclCommAbort returned %d after %.3f s\n", (int)ra, now_s() - a);
    aborted = true;
  });
  for (int k = 0; k < 40 && !aborted; k++) {
    std::this_thread::sleep_for(std::chrono::milliseconds(500));
    if (!aborted && (k % 4 == 1)) snapshot("while ncclCommAbort has not returned");
  }
  if (!aborted) {
    snapshot("abort still blocked after 20 s");
    fflush(stdout);
    _exit(2);
  }
  ab.join();
  printf("threads after abort %d\n", nthreads());
  snapshot("after abort");
  return 0;
}
