// Host check of the packet store layout (artis_amd/csrc/engine/packet_soa.h pkt_word_index): for a few packet counts
// n, the 38 payload words of every packet land on distinct words of the n * PKT_STORE_WORDS store; the words a line
// absorption writes (19, 21-24, 36, 37) share one 64-byte sector of the cold record, the words a deactivation
// writes (14-17, 25-30) lie in the record's two other sectors, and every packet's hot line and cold record start on
// a 64-byte boundary.  Built and run by tests/test_packet_layout.py.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "packet_soa.h"

int main() {
  long bad = 0;
  const int absorption[] = {19, 21, 22, 23, 24, 36, 37};
  const int deactivation[] = {14, 15, 16, 17, 25, 26, 27, 28, 29, 30};
  for (int64_t n : {1, 2, 3, 7, 64, 1000}) {
    std::vector<int> owner((size_t)n * PKT_STORE_WORDS, -1);
    for (int64_t i = 0; i < n; i++) {
      for (int w = 0; w < PKT_WORDS; w++) {
        const int64_t x = pkt_word_index(n, i, w);
        if (x < 0 || x >= n * PKT_STORE_WORDS || owner[x] != -1) {
          if (bad++ < 10) printf("clash: n %ld packet %ld word %d -> %ld\n", (long)n, (long)i, w, (long)x);
          continue;
        }
        owner[x] = w;
      }
      // hot line and cold record alignment (byte offsets of word 0 and of the cold record's first slot)
      if ((pkt_word_index(n, i, 0) * 8) % 128 != 0) bad++;
      const int64_t cold0 = 16 * n + i * PKT_COLD_WIDTH;
      if ((cold0 * 8) % 64 != 0) bad++;
      int64_t s0 = -1;
      for (int w : absorption) {
        const int64_t sec = (pkt_word_index(n, i, w) * 8) / 64;
        if (s0 < 0) s0 = sec;
        if (sec != s0 && bad++ < 10) printf("absorption word %d outside its sector (n %ld)\n", w, (long)n);
      }
      for (int w : deactivation) {
        const int64_t sec = (pkt_word_index(n, i, w) * 8) / 64;
        if ((sec == s0 || sec > s0 + 2) && bad++ < 10) printf("deactivation word %d in sector %ld (n %ld)\n", w,
                                                             (long)(sec - s0), (long)n);
      }
    }
  }
  printf("bad %ld\n", bad);
  return bad != 0;
}
