// CPU check of the grid-barrier launch sizing (kernels.h grid_barrier_grid), built host-only by
// tests/test_grid_barrier_cpu.py. Exit status 0 = every check passed.
#include <cstdio>

#include "kernels.h"

using smaml::grid_barrier_grid;

static int failures = 0;
#define CHECK(cond)                                                          \
  do {                                                                       \
    if (!(cond)) {                                                           \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      ++failures;                                                            \
    }                                                                        \
  } while (0)

int main() {
  // MI355X-like capacity: 256 CUs x 8 resident 256-thread blocks
  const int cap = 256 * 8;
  CHECK(grid_barrier_grid(cap, 64 * 5, 0) == 320);   // a 5-task group: one block per item
  CHECK(grid_barrier_grid(cap, 64 * 15, 0) == 512);  // 15 tasks: a quarter of the capacity
  CHECK(grid_barrier_grid(cap, 1, 0) == 1);
  // the grid never exceeds a quarter of the capacity, so four such grids are co-resident
  for (int items = 1; items < 100000; items = items * 3 + 1) {
    const int nb = grid_barrier_grid(cap, items, 0);
    CHECK(nb >= 1 && nb <= items && 4 * nb <= cap);
  }
  // tiny or partitioned devices
  CHECK(grid_barrier_grid(3, 100, 0) == 1);
  CHECK(grid_barrier_grid(8, 100, 0) == 2);
  // unknown capacity or nothing to do: 0 (the caller runs the two-launch form)
  CHECK(grid_barrier_grid(0, 100, 0) == 0);
  CHECK(grid_barrier_grid(-1, 100, 0) == 0);
  CHECK(grid_barrier_grid(cap, 0, 0) == 0);
  // debug oversize: strictly more blocks than can be resident
  CHECK(grid_barrier_grid(cap, 64, 1) == cap + 1);
  CHECK(grid_barrier_grid(cap, 64, 2) == 2 * cap + 1);
  if (failures) return 1;
  std::printf("grid_barrier_grid: all passed\n");
  return 0;
}
