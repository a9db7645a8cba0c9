// TOOLS / TESTS ONLY: the parallel pcap record walk (pcppx_pcap_map_batch / pcppx_pcap_read_batch_ex on regions of
// >= 4 MiB: interleaved chains per thread, starts kept across batches, parallel merge) over one capture with several
// batch sizes, the two calls alternating on one reader; prints packets and a checksum of the records per batch size
// (they must agree). tests/test_ingest.py builds it with -fsanitize=address,undefined.
//   ingest_parallel_check <capture>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "pcppx.h"
int main(int argc, char** argv) {
  const uint32_t sizes[] = {1u << 20, 70000, 333333};
  for (uint32_t B : sizes) {
    std::vector<uint64_t> off(B), ts(B); std::vector<uint32_t> cap(B), fl(B);
    pcppx_pcap* r; if (pcppx_pcap_open(argv[1], &r)) return 1;
    uint64_t np = 0, sum = 0;
    int alt = 0;
    std::vector<uint8_t> buf(64u << 20);
    for (;;) {
      uint32_t n = 0;
      if (alt++ & 1) {
        uint64_t used = 0;
        if (pcppx_pcap_read_batch_ex(r, buf.data(), buf.size(), off.data(), cap.data(), fl.data(), ts.data(), B, &n, &used)) return 3;
        for (uint32_t i = 0; i < n; ++i) sum += buf[off[i]] + cap[i];
      } else {
        const uint8_t* base; uint64_t sz;
        if (pcppx_pcap_map_batch(r, &base, &sz, off.data(), cap.data(), fl.data(), ts.data(), B, &n)) return 2;
        for (uint32_t i = 0; i < n; ++i) sum += base[off[i]] + cap[i];
      }
      if (!n) break;
      np += n;
    }
    pcppx_pcap_close(r);
    printf("batch %u: %llu packets, sum %llu\n", B, (unsigned long long)np, (unsigned long long)sum);
  }
}
