// getrow_bench.cpp -- C++-level GetRow latency through the product reader
// (okv_reader_get_row: btree floor, one host-mode decode of the block --
// the point path, okv_point_kernel -- row lookup), timed without Python.
// Beside it: the CPU restatement's decode of the same one block
// (oref_read_block from oracle/build/liboref.so, Go allocation semantics:
// a measurement baseline, dlopen'ed by this tool only) and the bloom-negative
// GetRow (host probe, no GPU call).
//
// build: tools/build_getrow_bench.sh   run: tools/getrow_bench [calls]
// prints one JSON line per block size.  Linked against the ablation build
// (tools/getrow_bench_ablate), it also prints the point kernel's phase
// times of one more GetRow (okv_debug_point_times: staged, walked,
// prefixes, emitted, in microseconds from the block's start).
#include <dlfcn.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "okv_host.h"
#include "okv_sst.h"

namespace {

typedef struct {
  uint8_t* key;
  uint64_t key_len;
  uint8_t* val;
  uint64_t val_len;
} oref_kv;
typedef struct {
  oref_kv* rows;
  uint64_t n, cap;
} oref_rows;
typedef int (*read_block_fn)(const uint8_t*, uint64_t, const okv_block_desc*, int, oref_rows*);
typedef void (*rows_free_fn)(oref_rows*);

double now_us() {
  return std::chrono::duration<double, std::micro>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

double pct(std::vector<double> v, double p) {
  std::sort(v.begin(), v.end());
  return v[std::min(v.size() - 1, size_t(p * double(v.size())))];
}

void key_of(uint64_t i, uint8_t* k) {  // OKV_SYNTH_FIXED: 8 zero bytes + big-endian index
  std::memset(k, 0, 8);
  for (int b = 0; b < 8; ++b) k[8 + b] = uint8_t(i >> (56 - 8 * b));
}

}  // namespace

int main(int argc, char** argv) {
  const int calls = argc > 1 ? std::atoi(argv[1]) : 2000;
  okv_ctx* ctx = okv_open(0);
  if (!ctx) {
    std::fprintf(stderr, "okv_open failed\n");
    return 1;
  }
  void* oref = dlopen("oracle/build/liboref.so", RTLD_NOW);
  read_block_fn oref_read = oref ? (read_block_fn)dlsym(oref, "oref_read_block") : nullptr;
  rows_free_fn oref_free = oref ? (rows_free_fn)dlsym(oref, "oref_rows_free") : nullptr;
  struct Cfg {
    const char* name;
    int kind;
    uint64_t rows, threshold, block;
  } cfgs[] = {{"4KiB_blocks", OKV_SYNTH_FIXED, 100000, 3584, 4096},
              {"64KiB_blocks", OKV_SYNTH_FIXED, 400000, 57344, 65536},
              // C3-shaped rows (Zipf key 8-256 B, value 0-4096 B): no two
              // neighbouring records need share a length; keys are the
              // blocks' FirstKeys (the row loop still walks the whole block)
              {"64KiB_zipf_blocks", OKV_SYNTH_ZIPF, 0, 57344, 65536}};
  for (const Cfg& c : cfgs) {
    okv_writer* w = c.kind == OKV_SYNTH_FIXED
                        ? okv_synth_segment(c.kind, 3, c.rows, 0, c.threshold, c.block)
                        : okv_synth_segment(c.kind, 3, 0, 600, c.threshold, c.block);
    uint64_t dlen = 0;  // (a closed writer)
    const uint8_t* data = okv_writer_data(w, &dlen);
    okv_reader* r = okv_reader_open(ctx, data, dlen, int64_t(dlen));
    if (okv_reader_fetch_metadata(r)) {
      std::fprintf(stderr, "metadata\n");
      return 1;
    }
    std::mt19937_64 rng(7);
    const uint64_t nblocks = okv_writer_num_blocks(w);
    uint8_t key[16];
    const uint8_t* kp = key;
    uint64_t kn = 16;
    auto pick = [&]() {  // a key of the segment
      if (c.kind == OKV_SYNTH_FIXED) {
        key_of(rng() % c.rows, key);
        kp = key;
        kn = 16;
      } else {
        okv_block_desc d;
        uint64_t h;
        okv_writer_block(w, rng() % nblocks, &d, &h, &kp, &kn);
      }
    };
    okv_row row;
    for (int i = 0; i < 50; ++i) {  // warm (slab allocation, code objects)
      pick();
      okv_reader_get_row(r, kp, kn, &row);
    }
    std::vector<double> t;
    okv_reader_io io0, io1;
    okv_reader_io_stats(r, &io0);
    for (int i = 0; i < calls; ++i) {
      pick();
      const double t0 = now_us();
      const int rc = okv_reader_get_row(r, kp, kn, &row);
      t.push_back(now_us() - t0);
      if (rc || row.key_len != kn || std::memcmp(row.key, kp, kn) != 0) {
        std::fprintf(stderr, "GetRow rc %d\n", rc);
        return 1;
      }
    }
    okv_reader_io_stats(r, &io1);
    typedef int (*times_fn)(uint64_t*);
    times_fn times = (times_fn)dlsym(RTLD_DEFAULT, "okv_debug_point_times");
    if (times) {
      double acc[4] = {0, 0, 0, 0};
      const int reps = 50;
      for (int i = 0; i < reps; ++i) {
        pick();
        okv_reader_get_row(r, kp, kn, &row);
        uint64_t t[5];
        times(t);
        for (int k = 0; k < 4; ++k) acc[k] += double(t[k + 1] - t[0]) / 100.0;
      }
      std::printf("{\"config\": \"%s\", \"point_phase_us\": {\"staged\": %.2f, \"walked\": %.2f, "
                  "\"prefixes\": %.2f, \"emitted\": %.2f}}\n",
                  c.name, acc[0] / reps, acc[1] / reps, acc[2] / reps, acc[3] / reps);
    }
    // the CPU restatement's one-block decode of the same blocks
    std::vector<double> tc;
    const uint64_t nb = nblocks;
    if (oref_read) {
      for (int i = 0; i < calls; ++i) {
        okv_block_desc d;
        uint64_t h, fl;
        const uint8_t* fk;
        okv_writer_block(w, rng() % nb, &d, &h, &fk, &fl);
        oref_rows rows{nullptr, 0, 0};
        const double t0 = now_us();
        oref_read(data, dlen, &d, 0, &rows);
        tc.push_back(now_us() - t0);
        oref_free(&rows);
      }
    }
    std::printf(
        "{\"config\": \"%s\", \"calls\": %d, \"gpu_calls\": %llu, \"blocks\": %llu, "
        "\"getrow_us\": {\"median\": %.1f, \"p90\": %.1f, \"p99\": %.1f, \"min\": %.1f}, "
        "\"cpu_restatement_one_block_us\": {\"median\": %.2f, \"p90\": %.2f}, "
        "\"path\": %u}\n",
        c.name, calls, (unsigned long long)(io1.calls - io0.calls),
        (unsigned long long)nb, pct(t, 0.5), pct(t, 0.9), pct(t, 0.99), pct(t, 0.0),
        tc.empty() ? -1.0 : pct(tc, 0.5), tc.empty() ? -1.0 : pct(tc, 0.9), okv_last_path(ctx));
    std::fflush(stdout);
    okv_reader_free(r);
    okv_writer_free(w);
  }
  okv_close(ctx);
  return 0;
}
