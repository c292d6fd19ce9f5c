// Bit-exact parallel evaluation of a sequential f64 sum
//     s = fl(...fl(fl(s0 + t_0) + t_1) ... + t_{n-1})
// -- the running sums of TEncoder.PrepareFrames (avgPower, totalPower,
// encoder.lpr:1374-1389), which the reference adds one sample at a time.
//
// While the running sum S stays inside one binade [2^e, 2^(e+1)), every
// partial sum is an integer multiple M of u = 2^(e-52) and
//     fl(M u + t) = (M + rnd(t / u)) u,
// where rnd rounds to the nearest integer, ties to the even RESULT M + r + {0,1}.
// t / u is exact (a power-of-two scaling), so a block of terms reduces to an
// integer sum of rounded increments plus the rare ties, whose choice needs the
// parity of M at that point.  A block is summarised in parallel under the
// binade a cheap approximate prefix predicts; the blocks are then chained in
// order, each in O(1 + ties), and a block whose summary does not apply (wrong
// binade guess, the sum leaves the binade inside it, S <= 0, huge or
// non-finite terms) is re-added term by term -- so the result is always the
// sequential one, bit for bit.  (The same argument as the yakmo prefix chain,
// gsc_yakmo.hip chain_fast, in f32.)
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <vector>

namespace gsc {

// floor of |q| < 2^52 without a libm call
inline double seqsum_floor(double q) {
    const double r = double(int64_t(q));
    return r > q ? r - 1.0 : r;
}

struct SeqSumStats {
    int64_t blocks = 0, fast_blocks = 0, ties = 0;
};

// fill(i0, i1, buf) writes t_{i0} .. t_{i1-1} into buf[0 .. i1-i0) (called with
// ranges of at most `block` terms, concurrently from the workers);
// parallel(nblocks, body) runs body(b) for b in [0, nblocks).
template <class FillFn, class ParFor>
double exact_seq_sum(int64_t n, double s0, const FillFn& fill, const ParFor& parallel, int64_t block = 8192,
                     SeqSumStats* stats = nullptr) {
    if (n <= 0) return s0;
    const int64_t nb = (n + block - 1) / block;
    struct Sum {
        double approx = 0.0;  // naive sum (binade prediction only)
        int e = 0;            // binade the summary assumes (ilogb of the block's start)
        bool ok = false;      // summary valid under e
        int64_t d = 0;        // sum of the rounded increments, ties rounded down
        int64_t pmin = 0, pmax = 0;  // extremes of the running prefix of those increments
        std::vector<int64_t> tie_pre;  // per tie: prefix of the increments before it (ties excluded)
    };
    std::vector<Sum> S(static_cast<size_t>(nb));
    std::vector<double> tb(static_cast<size_t>(block));  // the chaining loop's buffer
    parallel(int(nb), [&](int b) {
        const int64_t i0 = int64_t(b) * block, i1 = std::min(n, i0 + block);
        thread_local std::vector<double> buf;
        buf.resize(size_t(block));
        fill(i0, i1, buf.data());
        double a = 0.0;
        for (int64_t i = 0; i < i1 - i0; ++i) a += buf[size_t(i)];
        S[size_t(b)].approx = a;
        // the summary under the binade the block would have if the approximate
        // prefix were exact is computed below, once that prefix is known
    });
    // predicted binade of every block: both ends of the approximate prefix in
    // one binade (a wrong guess only costs the block a term-by-term pass)
    {
        double a = s0;
        for (int64_t b = 0; b < nb; ++b) {
            const double lo = a, hi = a + S[size_t(b)].approx;
            a = hi;
            Sum& s = S[size_t(b)];
            s.ok = false;
            if (!(lo > 0.0) || !(hi > 0.0) || !std::isfinite(lo) || !std::isfinite(hi)) continue;
            const int e = std::ilogb(lo);
            if (std::ilogb(hi) != e || e < -1000 || e > 1000) continue;
            s.e = e;
            s.ok = true;
        }
    }
    parallel(int(nb), [&](int b) {
        Sum& s = S[size_t(b)];
        if (!s.ok) return;
        const int64_t i0 = int64_t(b) * block, i1 = std::min(n, i0 + block);
        thread_local std::vector<double> buf;
        buf.resize(size_t(block));
        fill(i0, i1, buf.data());
        const double scale = std::ldexp(1.0, 52 - s.e);  // 1 / u
        int64_t p = 0, pmin = 0, pmax = 0;
        for (int64_t i = 0; i < i1 - i0; ++i) {
            const double q = buf[size_t(i)] * scale;  // t / u, exact unless it leaves the normal range
            if (!(std::fabs(q) < 0x1p52) || (q != 0.0 && std::fabs(q) < 0x1p-1000)) {  // add term by term
                s.ok = false;
                return;
            }
            const double r = seqsum_floor(q), f = q - r;  // both exact
            if (f == 0.5) {
                s.tie_pre.push_back(p);
                p += int64_t(r);
            } else {
                p += int64_t(r) + (f > 0.5 ? 1 : 0);
            }
            pmin = std::min(pmin, p);
            pmax = std::max(pmax, p);
        }
        s.d = p;
        s.pmin = pmin;
        s.pmax = pmax;
    });
    double acc = s0;
    for (int64_t b = 0; b < nb; ++b) {
        const Sum& s = S[size_t(b)];
        const int64_t i0 = b * block, i1 = std::min(n, i0 + block);
        bool fast = s.ok && acc > 0.0 && std::isfinite(acc) && std::ilogb(acc) == s.e;
        int64_t M0 = 0;
        const int64_t nt = int64_t(s.tie_pre.size());
        if (fast) {
            M0 = int64_t(std::ldexp(acc, 52 - s.e));  // exact integer in [2^52, 2^53)
            // every running sum (ties adding 0 or 1 each) must stay strictly inside the binade
            fast = M0 + s.pmin - nt >= (int64_t(1) << 52) + 1 && M0 + s.pmax + nt <= (int64_t(1) << 53) - 2;
        }
        if (stats) ++stats->blocks;
        if (!fast) {
            fill(i0, i1, tb.data());
            for (int64_t i = 0; i < i1 - i0; ++i) acc = acc + tb[size_t(i)];
            continue;
        }
        if (stats) {
            ++stats->fast_blocks;
            stats->ties += nt;
        }
        // ties in order: the rounded-down candidate M0 + pre + added (+ r, folded into pre's
        // successor) -- pick the even result
        int64_t added = 0;
        if (nt > 0) {
            // re-walk the block's ties: the candidate below a tie is M0 + tie_pre + added + floor(q)
            const double scale = std::ldexp(1.0, 52 - s.e);
            fill(i0, i1, tb.data());
            int64_t k = 0;
            for (int64_t i = 0; i < i1 - i0 && k < nt; ++i) {
                const double q = tb[size_t(i)] * scale;
                const double r = seqsum_floor(q);
                if (q - r != 0.5) continue;
                const int64_t below = M0 + s.tie_pre[size_t(k)] + added + int64_t(r);
                if (below & 1) ++added;  // ties to even
                ++k;
            }
        }
        acc = std::ldexp(double(M0 + s.d + added), s.e - 52);
    }
    return acc;
}

}  // namespace gsc
