// Scheduler of the host-side SIMT emulator (see include/hip/hip_runtime.h).
// TEST INFRASTRUCTURE ONLY: linked with the product's csrc/*.hip compiled as
// host C++ into tests/emu/_build/libgd_emu.so.
#include <hip/hip_runtime.h>

#include <sys/mman.h>

#include <algorithm>
#include <random>

// bounds of the LDS section (include/hip/hip_runtime.h: __shared__)
extern "C" char __start_gd_emu_lds[] __attribute__((weak));
extern "C" char __stop_gd_emu_lds[] __attribute__((weak));

namespace gd_emu {
namespace {

constexpr size_t kStack = 256 * 1024;

Grid g_grid;
std::vector<void*> g_stacks;  // reused across launches (mmap'd, touched lazily)
uint64_t g_progress = 0;      // bumped by every publish / arrival / exit

void* stack_for(size_t i) {
  while (g_stacks.size() <= i) {
    void* p = mmap(nullptr, kStack, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p == MAP_FAILED) {
      perror("gd_emu: mmap");
      abort();
    }
    g_stacks.push_back(p);
  }
  return g_stacks[i];
}

void release_if_complete() {
  Grid& g = g_grid;
  if (g.arrived > 0 && g.arrived == g.live) {
    g.arrived = 0;
    ++g.gen;
  }
}

enum class Sched { kFwd, kRev, kShuffle };
Sched g_sched = Sched::kFwd;
std::mt19937 g_rng;

void read_sched_env() {
  static bool done = false;
  if (done) return;
  done = true;
  const char* e = getenv("GD_EMU_SCHED");
  if (!e || !*e || !strcmp(e, "fwd")) return;
  if (!strcmp(e, "rev")) {
    g_sched = Sched::kRev;
  } else if (!strncmp(e, "shuffle:", 8)) {
    g_sched = Sched::kShuffle;
    g_rng.seed(unsigned(strtoul(e + 8, nullptr, 10)));
  } else {
    fprintf(stderr, "gd_emu: GD_EMU_SCHED=%s (want fwd | rev | shuffle:<seed>)\n", e);
    abort();
  }
}

void poison_lds() {
  if (+__start_gd_emu_lds && +__stop_gd_emu_lds && +__stop_gd_emu_lds > +__start_gd_emu_lds)
    memset(__start_gd_emu_lds, 0xFF, size_t(__stop_gd_emu_lds - __start_gd_emu_lds));
}

void trampoline() {
  Grid& g = g_grid;
  g.body(g.body_arg);
  Item& me = g.items[g.cur];
  me.done = true;
  --g.live;
  ++g_progress;
  release_if_complete();
  // returning resumes uc_link (the scheduler)
}

}  // namespace

Grid& grid() { return g_grid; }

void note_progress() { ++g_progress; }

void yield() {
  Grid& g = g_grid;
  swapcontext(&g.items[g.cur].ctx, &g.sched);
}

void syncthreads() {
  Grid& g = g_grid;
  const unsigned gen = g.gen;
  ++g.arrived;
  ++g_progress;
  release_if_complete();
  while (g.gen == gen) yield();
}

void run(dim3 gd, dim3 bd, void (*body)(void*), void* arg) {
  Grid& g = g_grid;
  const unsigned n = bd.x * bd.y * bd.z;
  if (n == 0 || n > 1024 || gd.x == 0 || gd.y == 0 || gd.z == 0) {
    fprintf(stderr, "gd_emu: bad launch grid (%u,%u,%u) block (%u,%u,%u)\n", gd.x, gd.y, gd.z, bd.x, bd.y, bd.z);
    abort();
  }
  g.grid = gd;
  g.block = bd;
  g.body = body;
  g.body_arg = arg;
  g.items.resize(n);
  read_sched_env();
  std::vector<unsigned> order(n);
  for (unsigned i = 0; i < n; ++i) order[i] = g_sched == Sched::kRev ? n - 1 - i : i;
  for (unsigned bz = 0; bz < gd.z; ++bz)
    for (unsigned by = 0; by < gd.y; ++by)
      for (unsigned bx = 0; bx < gd.x; ++bx) {
        g.bid = dim3(bx, by, bz);
        for (unsigned i = 0; i < n; ++i) {
          Item& it = g.items[i];
          it.tid = dim3(i % bd.x, (i / bd.x) % bd.y, i / (bd.x * bd.y));
          it.done = false;
          it.nxchg = 0;
          it.published.clear();
          getcontext(&it.ctx);
          it.ctx.uc_stack.ss_sp = stack_for(i);
          it.ctx.uc_stack.ss_size = kStack;
          it.ctx.uc_link = &g.sched;
          makecontext(&it.ctx, trampoline, 0);
        }
        g.live = n;
        g.arrived = 0;
        poison_lds();
        while (g.live > 0) {
          const uint64_t before = g_progress;
          if (g_sched == Sched::kShuffle) std::shuffle(order.begin(), order.end(), g_rng);
          for (unsigned i : order) {
            if (g.items[i].done) continue;
            g.cur = i;
            swapcontext(&g.sched, &g.items[i].ctx);
          }
          if (g_progress == before && g.live > 0) {
            fprintf(stderr, "gd_emu: deadlock in block (%u,%u,%u): %u work-items wait forever\n", bx, by, bz,
                    g.live);
            abort();
          }
        }
      }
}

}  // namespace gd_emu
