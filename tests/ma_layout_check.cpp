// Host check of the macro-atom key-record layout (artis_amd/csrc/engine/engine_dev.h ma_layout / ma_rec_pos) and of
// the search k_ma makes over it (transport.h ma_step_cached): for every (nd, nu) shape the layout accepts, every
// record position is written at most once, line-0 copies stay on line 0, and for every entry j of the down-same and
// up-same arrays a draw just below key j is resolved to j by the line-0 search of the block separators and suffix,
// then (if it names a block) the search of that block line.  Built and run by tests/test_ma_layout.py.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#include "engine_dev.h"

int main() {
  long bad = 0, checked = 0, shapes = 0;
  for (int nd = 0; nd <= 300; nd++)
    for (int nu = 0; nu <= 700; nu += (nu < 130 ? 1 : 7)) {
      if (!ma_layout_ok(nd, nu)) continue;
      shapes++;
      const int nr = 3, nt = 2;
      const MaLayout L = ma_layout(nd, nu, nr, nt);
      const int len = 9 + 2 * nd + nu + 2 * nr + nt;
      std::vector<int> owner(L.hot, -1);  // the scratch position stored at each record position
      for (int p = 0; p < len; p++) {
        int sp;
        const int rp = ma_rec_pos(L, p, nd, nu, &sp);
        if (rp < 0 || rp >= L.hot || owner[rp] != -1) {
          if (bad++ < 10) printf("position clash: nd %d nu %d p %d -> %d\n", nd, nu, p, rp);
          break;
        }
        owner[rp] = p;
        if (sp >= 0) {
          if (sp >= 64 || owner[sp] != -1) {
            if (bad++ < 10) printf("separator clash: nd %d nu %d p %d -> %d\n", nd, nu, p, sp);
            break;
          }
          owner[sp] = p;
        }
      }
      for (int arr = 0; arr < 2; arr++) {
        const int c = arr ? nu : nd, nb = arr ? L.nbu : L.nbd, suf = arr ? L.mu : L.md, a0 = arr ? 9 + L.sd : 9;
        const int p0 = arr ? 9 + nd : 9;
        auto key = [&](int pos) { return owner[pos] - p0 + 1; };  // entry j's running sum is j + 1
        for (int q = 0; q < c; q++) {  // a draw in [j, j + 1) selects entry j = q
          checked++;
          const int end = nb ? ma_nsep(nb) + suf : c;
          int lo = 0, hi = end;
          while (lo < hi) {
            const int mid = (lo + hi) / 2;
            if (key(a0 + mid) > q) hi = mid; else lo = mid + 1;
          }
          int j;
          if (nb && lo < nb) {
            const int base = 64 * (1 + (arr ? L.nbd : 0) + lo), e = std::min(64, c - suf - 64 * lo);
            int l2 = 0, h2 = e;
            while (l2 < h2) {
              const int mid = (l2 + h2) / 2;
              if (key(base + mid) > q) h2 = mid; else l2 = mid + 1;
            }
            j = l2 < e ? 64 * lo + l2 : -1;
          } else {
            j = lo < end ? (nb ? c - suf + lo - nb : lo) : -1;
          }
          if (j != q && bad++ < 10) printf("search: nd %d nu %d array %d draw %d -> %d\n", nd, nu, arr, q, j);
        }
      }
    }
  printf("shapes %ld searches %ld bad %ld\n", shapes, checked, bad);
  return bad ? 1 : 0;
}
