// Concurrency stress driver for the native volume reader (csrc/runtime/volume_io_core.h), built and run on the
// host with ThreadSanitizer and with AddressSanitizer+UBSan by tests/test_cpu_runtime.py (race detection for
// the runtime's worker pool, ticket registry and completion signalling; the reference has none).
//
//   volume_io_stress <dir> [submitters] [rounds]
//
// Writes a small NIDTVOL1 file whose voxel bytes encode (subject, offset), then several host threads submit
// overlapping asynchronous gathers, poll done(), wait and verify every byte; a final reader is destroyed
// with gathers still queued (the destructor must drain them before unmapping).
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <random>

#include "../volume_io_core.h"

using nidt_io::Header;
using nidt_io::VolumeReader;

static uint8_t expect(int64_t s, size_t i) { return (uint8_t)((s * 131 + i * 7 + (i >> 9)) & 0xff); }

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s <dir> [submitters] [rounds]\n", argv[0]);
    return 2;
  }
  const std::string path = std::string(argv[1]) + "/stress.nidtvol";
  const int nsub = argc > 2 ? std::atoi(argv[2]) : 4, rounds = argc > 3 ? std::atoi(argv[3]) : 40;
  const uint64_t N = 23, D = 37, H = 41, W = 29, vox = D * H * W;  // vox not a multiple of the 1 MiB piece
  {
    Header h{};
    std::memcpy(h.magic, "NIDTVOL1", 8);
    h.version = 1;
    h.dtype = 0;
    h.n = N; h.d = D; h.h = H; h.w = W;
    h.data_off = 4096;
    h.labels_off = h.data_off + N * vox;
    h.sites_off = h.labels_off + 4 * N;
    std::ofstream f(path, std::ios::binary);
    f.write(reinterpret_cast<const char*>(&h), sizeof(h));
    std::vector<char> pad(h.data_off - sizeof(h), 0);
    f.write(pad.data(), pad.size());
    std::vector<uint8_t> v(vox);
    for (uint64_t s = 0; s < N; ++s) {
      for (size_t i = 0; i < vox; ++i) v[i] = expect((int64_t)s, i);
      f.write(reinterpret_cast<const char*>(v.data()), vox);
    }
    for (uint64_t s = 0; s < 2 * N; ++s) {
      const float x = (float)(s % N);
      f.write(reinterpret_cast<const char*>(&x), 4);
    }
  }
  std::atomic<int> bad{0};
  {
    VolumeReader r(path, 6);
    std::vector<float> lab(N);
    r.copy_labels(lab.data());
    if (r.n() != N || r.voxels() != vox || lab[5] != 5.f) {
      std::fprintf(stderr, "header mismatch\n");
      return 1;
    }
    std::vector<std::thread> th;
    for (int t = 0; t < nsub; ++t) {
      th.emplace_back([&, t] {
        std::mt19937 rng(1234 + t);
        for (int it = 0; it < rounds; ++it) {
          const int k = 1 + (int)(rng() % 5);
          std::vector<int64_t> ix(k);
          for (auto& s : ix) s = (int64_t)(rng() % N);
          std::vector<uint8_t> buf(k * vox, 0xAB);
          const int64_t id = r.submit(ix, reinterpret_cast<uintptr_t>(buf.data()));
          if (it & 1) {
            while (!r.done(id)) std::this_thread::yield();
          }
          r.wait(id);
          if (it % 7 == 3) r.prefetch(ix);
          for (int j = 0; j < k; ++j)
            for (size_t i = 0; i < vox; i += 97)
              if (buf[j * vox + i] != expect(ix[j], i)) {
                bad.fetch_add(1);
                break;
              }
          std::vector<uint8_t> b2(vox);
          r.gather({ix[0]}, reinterpret_cast<uintptr_t>(b2.data()));
          if (b2[vox - 1] != expect(ix[0], vox - 1)) bad.fetch_add(1);
        }
      });
    }
    for (auto& x : th) x.join();
  }
  {  // destroy with work still queued
    std::vector<uint8_t> buf(8 * vox);
    {
      VolumeReader r(path, 2);
      std::vector<int64_t> ix = {0, 1, 2, 3, 4, 5, 6, 7};
      r.submit(ix, reinterpret_cast<uintptr_t>(buf.data()));
    }
    for (int j = 0; j < 8; ++j)
      if (buf[j * vox + 11] != expect(j, 11)) bad.fetch_add(1);
  }
  bool threw = false;
  try {
    VolumeReader r(path, 1);
    r.submit({(int64_t)N}, 1);
  } catch (const std::out_of_range&) {
    threw = true;
  }
  std::remove(path.c_str());
  if (bad.load() || !threw) {
    std::fprintf(stderr, "FAIL bad=%d threw=%d\n", bad.load(), (int)threw);
    return 1;
  }
  std::printf("volume_io_stress ok (%d submitters x %d rounds)\n", nsub, rounds);
  return 0;
}
