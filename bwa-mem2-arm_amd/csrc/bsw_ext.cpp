// bsw_ext.cpp -- seed-extension job builder + result interpreter (include/bsw_ext.h).
//
// Host C++ around the batch engine, restating the extension half of upstream's
// mem_chain2aln / mem_chain2aln_across_reads_V2 (src/bwamem.cpp; semantics in bsw_ext.h and
// SURVEY.md a9/§8(f) row 1).  Per call:
//   phase 0  LEFT  jobs (qbeg > 0): reversed query prefix vs reversed target window, h0 = seed
//            score, band w; phase 1: LEFT retries with w << 1 where the score changed and
//            max_off >= 3/4 w (MAX_BAND_TRY); interpret local vs to-end with pen_clip5
//   phase 2  RIGHT jobs (qe < l_query): query suffix vs target window, h0 = the LEFT score;
//            phase 3: retries; interpret with pen_clip3
// Each phase is ONE bsw batch over all reads (SeqPair AoS + concatenated code buffers in
// upstream's layout); buffers are filled by a host thread pool.  The CPU restatement used as
// the oracle is oracle/ext_ref.c.
#include <algorithm>
#include <chrono>
#include <cstring>
#include <memory>
#include <thread>
#include <vector>
#include "../../include/bsw_ext.h"
#include "bsw_internal.h"
#include "bsw_pool.h"

namespace {

using Clock = std::chrono::steady_clock;
float ms_since(Clock::time_point t0)
{
    return std::chrono::duration<float, std::milli>(Clock::now() - t0).count();
}

struct Job {                       // one extension of one read
    int32_t read;                  // read index
    int32_t qlen, tlen;
    int64_t qoff, toff;            // offsets into the phase's code buffers
};

int cal_max_gap(const bsw_params_t &p, int a, int w, int qlen)
{
    const int l_del = (int)((double)(qlen * a - p.o_del) / p.e_del + 1.);
    const int l_ins = (int)((double)(qlen * a - p.o_ins) / p.e_ins + 1.);
    int l = std::max(l_del, l_ins);
    l = std::max(l, 1);
    return std::min(l, w << 1);
}

// mem_chain2aln's target window of a chain (include/bsw_ext.h; oracle_chain_window): min / max
// of the seeds' reach, clipped to [0, ref_len), and with l_pac > 0 the side of the first seed
// when it crosses the forward-reverse boundary.  seed(i) returns the chain's i-th seed.
template <class Seed>
void chain_window(const bsw_params_t &p, int a, const bsw_ext_opt_t &opt, int64_t ref_len, int l_query, int n,
                  Seed seed, int64_t *rmax0, int64_t *rmax1)
{
    int64_t lo = ref_len, hi = 0, first = -1;
    for (int i = 0; i < n; ++i) {
        const bsw_seed_t &t = seed(i);
        if (t.len <= 0) continue;
        if (first < 0) first = t.rbeg;
        const int32_t qe = t.qbeg + t.len;
        lo = std::min<int64_t>(lo, t.rbeg - (t.qbeg + cal_max_gap(p, a, opt.w, t.qbeg)));
        hi = std::max<int64_t>(hi, t.rbeg + t.len + ((l_query - qe) + cal_max_gap(p, a, opt.w, l_query - qe)));
    }
    lo = std::max<int64_t>(lo, 0);
    hi = std::min<int64_t>(hi, ref_len);
    if (opt.l_pac > 0 && lo < opt.l_pac && opt.l_pac < hi) {
        if (first < opt.l_pac) hi = opt.l_pac;
        else lo = opt.l_pac;
    }
    *rmax0 = lo;
    *rmax1 = hi;
}

// f(a, b) over [0, n) in pieces on the engine's host pool (bsw_pool.h)
template <class F>
void parallel_for(int32_t n, F f)
{
    const int nt = bsw::HostPool::workers() + 1;
    if (n < 4096) {
        f(0, n);
        return;
    }
    bsw::HostPool::get().parallel_for(nt, [&](int t) {
        f((int32_t)((int64_t)n * t / nt), (int32_t)((int64_t)n * (t + 1) / nt));
    });
}

struct Buf {                       // code buffer: pinned per-context staging when free, else heap
    bsw_ctx_t *ctx = nullptr;
    int which = 0;
    uint8_t *p = nullptr;
    bool pinned = false;
    std::unique_ptr<uint8_t[]> heap;
    void get(bsw_ctx_t *c, int w, size_t bytes)
    {
        ctx = c; which = w;
        p = (uint8_t *)bsw::pinned_acquire(c, w, bytes);
        pinned = p != nullptr;
        if (!pinned) { heap.reset(new uint8_t[bytes]); p = heap.get(); }   // uninitialised
    }
    ~Buf() { if (pinned) bsw::pinned_release(ctx, which); }
};

struct Phase {                     // one batch: jobs + SeqPairs + code buffers
    std::vector<Job> jobs;
    std::vector<SeqPair> pairs;
    Buf qbuf, tbuf;

    // lay out buffers for jobs (qlen/tlen set), fill with `fill(job, qdst, tdst)`
    template <class Fill>
    void build(bsw_ctx_t *ctx, Fill fill)
    {
        int64_t qo = 0, to = 0;
        for (auto &j : jobs) {
            j.qoff = qo; j.toff = to;
            qo += j.qlen; to += j.tlen;
        }
        qbuf.get(ctx, 0, (size_t)std::max<int64_t>(qo, 1));
        tbuf.get(ctx, 1, (size_t)std::max<int64_t>(to, 1));
        pairs.resize(jobs.size());
        parallel_for((int32_t)jobs.size(), [&](int32_t a, int32_t b) {
            for (int32_t k = a; k < b; ++k) {
                const Job &j = jobs[k];
                fill(j, qbuf.p + j.qoff, tbuf.p + j.toff);
                SeqPair &p = pairs[k];
                p = SeqPair{};
                p.idr = (int32_t)j.toff; p.idq = (int32_t)j.qoff;
                p.id = j.read; p.len1 = j.tlen; p.len2 = j.qlen;
            }
        });
    }
};

}  // namespace

extern "C" void bsw_ext_opt_default(bsw_ext_opt_t *opt)
{
    opt->w = 100;
    opt->pen_clip5 = 5;
    opt->pen_clip3 = 5;
    opt->max_band_try = 2;
    opt->l_pac = 0;
}

namespace bsw {

int ext_opt_check(const bsw_ext_opt_t *opt, int64_t ref_len)
{
    if (opt->w < 0 || opt->max_band_try < 1 || ref_len < 0 || opt->l_pac < 0) return BSW_E_INVAL;
    if (opt->l_pac > 0 && ref_len != 2 * opt->l_pac) return BSW_E_INVAL;
    return BSW_OK;
}

// a seed must lie inside [0, ref_len) and, on a two-strand text, on one strand (upstream's
// bns_intv2rid drops bridging seeds before chaining)
bool ext_seed_ok(const bsw_ext_opt_t *opt, const bsw_seed_t &s, int32_t l, int64_t ref_len)
{
    if (s.qbeg < 0 || s.qbeg + s.len > l || s.rbeg < 0 || s.rbeg + s.len > ref_len || l > BSW_MAX_LEN) return false;
    return !(opt->l_pac > 0 && s.rbeg < opt->l_pac && s.rbeg + s.len > opt->l_pac);
}

}  // namespace bsw

extern "C" int bsw_ext_last_stats(bsw_ctx_t *ctx, bsw_ext_stats_t *out)
{
    return bsw::get_ext_stats(ctx, out);
}

// The extension of n seeds, seed i inside the target window win[2i], win[2i + 1] (a chain's
// window, mem_chain2aln) or, with win == nullptr, its own one-seed window.
static int extend_seeds_win(bsw_ctx_t *ctx, const bsw_ext_opt_t *opt, const uint8_t *ref, int64_t ref_len,
                            const uint8_t *reads, const int64_t *read_off, const int32_t *read_len,
                            const bsw_seed_t *seeds, const int64_t *win, int32_t n, bsw_alnreg_t *out)
{
    if (!ctx || !opt || n < 0 || (n > 0 && (!ref || !reads || !read_off || !read_len || !seeds || !out)))
        return BSW_E_INVAL;
    if (const int rc = bsw::ext_opt_check(opt, ref_len)) return rc;
    // SeqPair idr / idq are int32 offsets into one phase's code buffers: split calls whose
    // buffers could pass 2^31 bytes (window <= read + 2 cal_max_gap <= read + 4w per read)
    {
        int64_t maxlen = 0;
        for (int32_t i = 0; i < n; ++i) maxlen = std::max<int64_t>(maxlen, read_len[i]);
        const int64_t per_read = maxlen + ((int64_t)opt->w << 2) + 2;
        int64_t chunk = std::max<int64_t>(1, (int64_t)INT32_MAX / per_read - 1);
        chunk = std::min<int64_t>(chunk, bsw::ext_chunk_cap(ctx));  // BSW_OPT_EXT_CHUNK
        if (n > chunk) {
            bsw_ext_stats_t agg{};
            for (int64_t a0 = 0; a0 < n; a0 += chunk) {
                const int32_t m = (int32_t)std::min<int64_t>(chunk, n - a0);
                const int rc = extend_seeds_win(ctx, opt, ref, ref_len, reads, read_off + a0, read_len + a0,
                                                seeds + a0, win ? win + 2 * a0 : nullptr, m, out + a0);
                if (rc) return rc;
                bsw_ext_stats_t st{};
                bsw::get_ext_stats(ctx, &st);
                for (int k = 0; k < 4; ++k) agg.n_pairs[k] += st.n_pairs[k];
                agg.kernel_ms += st.kernel_ms; agg.build_ms += st.build_ms;
                agg.engine_ms += st.engine_ms; agg.interp_ms += st.interp_ms;
            }
            bsw::set_ext_stats(ctx, agg);
            return BSW_OK;
        }
    }
    bsw_params_t p;
    bsw::ctx_params(ctx, &p);
    const int a = p.mat[0];
    bsw_ext_stats_t es{};
    // per-read state (mem_alnreg_t subset + the window and scores the phases need)
    std::vector<int64_t> rmax0(n), rmax1(n);
    std::vector<int32_t> score(n, 0), lw(n, opt->w), rw(n, opt->w);   // aw[0], aw[1]
    for (int32_t i = 0; i < n; ++i) {
        bsw_alnreg_t &r = out[i];
        memset(&r, 0, sizeof(r));
        const bsw_seed_t &s = seeds[i];
        if (s.len <= 0) continue;
        const int32_t l = read_len[i];
        if (!bsw::ext_seed_ok(opt, s, l, ref_len)) return BSW_E_RANGE;
        if (win) {
            rmax0[i] = win[2 * i];
            rmax1[i] = win[2 * i + 1];
        } else {
            chain_window(p, a, *opt, ref_len, l, 1, [&](int) -> const bsw_seed_t & { return s; }, &rmax0[i],
                         &rmax1[i]);
        }
        if (rmax0[i] > s.rbeg || rmax1[i] < s.rbeg + s.len || s.rbeg - rmax0[i] > BSW_MAX_LEN ||
            rmax1[i] - (s.rbeg + s.len) > BSW_MAX_LEN)
            return BSW_E_RANGE;
        r.seedlen0 = s.len;
        // no-extension defaults (mem_chain2aln): qbeg == 0 / qe == l_query
        r.score = r.truesc = s.len * a;
        r.qb = 0; r.rb = s.rbeg;
        r.qe = l; r.re = s.rbeg + s.len;
        score[i] = s.len * a;
    }

    // run one side: build jobs, batch (+ retries), return per-job final SeqPair and band
    auto run_side = [&](bool left, int phase0, std::vector<int32_t> &band) -> int {
        auto tb = Clock::now();
        Phase ph;
        ph.jobs.reserve((size_t)n);
        for (int32_t i = 0; i < n; ++i) {
            const bsw_seed_t &s = seeds[i];
            if (s.len <= 0) continue;
            const int32_t qe = s.qbeg + s.len;
            if (left ? s.qbeg == 0 : qe == read_len[i]) continue;
            Job j{};
            j.read = i;
            j.qlen = left ? s.qbeg : read_len[i] - qe;
            j.tlen = left ? (int32_t)(s.rbeg - rmax0[i]) : (int32_t)(rmax1[i] - (s.rbeg + s.len));
            ph.jobs.push_back(j);
        }
        if (ph.jobs.empty()) return BSW_OK;
        ph.build(ctx, [&](const Job &j, uint8_t *qd, uint8_t *td) {
            const bsw_seed_t &s = seeds[j.read];
            const uint8_t *q = reads + read_off[j.read];
            if (left) {             // reversed prefix / reversed window ending at rbeg
                for (int32_t k = 0; k < j.qlen; ++k) qd[k] = q[s.qbeg - 1 - k];
                for (int32_t k = 0; k < j.tlen; ++k) td[k] = ref[s.rbeg - 1 - k];
            } else {
                memcpy(qd, q + s.qbeg + s.len, (size_t)j.qlen);
                memcpy(td, ref + s.rbeg + s.len, (size_t)j.tlen);
            }
        });
        const int32_t nj = (int32_t)ph.jobs.size();
        std::vector<int32_t> prev(nj);
        for (int32_t k = 0; k < nj; ++k) {
            const int32_t i = ph.jobs[k].read;
            ph.pairs[k].h0 = left ? seeds[i].len * a : score[i];
            prev[k] = left ? 0 : score[i];     // a->score before the band loop
            band[i] = opt->w;
        }
        const int32_t eb = left ? opt->pen_clip5 : opt->pen_clip3;
        es.build_ms += ms_since(tb);
        auto te = Clock::now();
        bsw_stats_t st{};
        int rc = bsw::scores_eb(ctx, eb, ph.pairs.data(), ph.tbuf.p, ph.qbuf.p, nj, opt->w, 16, &st);
        if (rc) return rc;
        es.n_pairs[phase0] += nj;
        es.kernel_ms += st.kernel_ms;
        // band retries: score changed and max_off >= 3/4 of the band -> redo with w << t
        std::vector<int32_t> idx(nj);
        for (int32_t k = 0; k < nj; ++k) idx[k] = k;
        for (int t = 1; t < opt->max_band_try; ++t) {
            const int32_t wt = opt->w << (t - 1), wn = opt->w << t;
            std::vector<int32_t> redo;
            for (int32_t k : idx) {
                const SeqPair &sp = ph.pairs[k];
                if (!(sp.score == prev[k] || sp.max_off < (wt >> 1) + (wt >> 2))) redo.push_back(k);
            }
            if (redo.empty()) break;
            std::vector<SeqPair> sub(redo.size());
            for (size_t r = 0; r < redo.size(); ++r) {
                prev[redo[r]] = ph.pairs[redo[r]].score;
                sub[r] = ph.pairs[redo[r]];
            }
            rc = bsw::scores_eb(ctx, eb, sub.data(), ph.tbuf.p, ph.qbuf.p, (int32_t)sub.size(), wn,
                                16, &st);
            if (rc) return rc;
            es.n_pairs[phase0 + 1] += (int32_t)sub.size();
            es.kernel_ms += st.kernel_ms;
            for (size_t r = 0; r < redo.size(); ++r) {
                ph.pairs[redo[r]] = sub[r];
                band[ph.jobs[redo[r]].read] = wn;
            }
            idx = redo;
        }
        es.engine_ms += ms_since(te);
        auto ti = Clock::now();
        // interpret (mem_chain2aln local vs to-end)
        for (int32_t k = 0; k < nj; ++k) {
            const SeqPair &sp = ph.pairs[k];
            const int32_t i = ph.jobs[k].read;
            const bsw_seed_t &s = seeds[i];
            bsw_alnreg_t &r = out[i];
            if (left) {
                r.score = sp.score;
                if (sp.gscore <= 0 || sp.gscore <= sp.score - opt->pen_clip5) {
                    r.qb = s.qbeg - sp.qle; r.rb = s.rbeg - sp.tle; r.truesc = sp.score;
                } else {
                    r.qb = 0; r.rb = s.rbeg - sp.gtle; r.truesc = sp.gscore;
                }
                score[i] = sp.score;
            } else {
                const int32_t sc0 = score[i];
                const int32_t qe = s.qbeg + s.len;
                r.score = sp.score;
                if (sp.gscore <= 0 || sp.gscore <= sp.score - opt->pen_clip3) {
                    r.qe = qe + sp.qle; r.re = s.rbeg + s.len + sp.tle; r.truesc += sp.score - sc0;
                } else {
                    r.qe = read_len[i]; r.re = s.rbeg + s.len + sp.gtle; r.truesc += sp.gscore - sc0;
                }
                score[i] = sp.score;
            }
        }
        es.interp_ms += ms_since(ti);
        return BSW_OK;
    };
    int rc = run_side(true, 0, lw);
    if (rc) return rc;
    rc = run_side(false, 2, rw);
    if (rc) return rc;
    for (int32_t i = 0; i < n; ++i)
        if (seeds[i].len > 0) out[i].w = std::max(lw[i], rw[i]);
    bsw::set_ext_stats(ctx, es);
    return BSW_OK;
}

extern "C" int bsw_extend_seeds(bsw_ctx_t *ctx, const bsw_ext_opt_t *opt, const uint8_t *ref,
                                int64_t ref_len, const uint8_t *reads, const int64_t *read_off,
                                const int32_t *read_len, const bsw_seed_t *seeds, int32_t n,
                                bsw_alnreg_t *out)
{
    return extend_seeds_win(ctx, opt, ref, ref_len, reads, read_off, read_len, seeds, nullptr, n, out);
}

// ---------------------------------------------------------------- mem_chain2aln over chains
// The per-read order of upstream's mem_chain2aln (chains in order, each chain's seeds by score
// descending; a seed contained "around" an earlier region of the read is skipped unless an
// extended, >= 95%-as-long seed of its chain overlaps it off-diagonal; SURVEY.md §8(f) row 1,
// oracle/ext_ref.c oracle_chain2aln) run ACROSS reads in rounds: round r extends, for every
// read, the next seed its containment test keeps -- one LEFT + RIGHT batch set per round
// (mem_chain2aln_across_reads_V2's batching), so only the skip decisions are sequential per
// read.  Rounds <= seeds per read; most reads finish in round 1 (their later seeds fall
// inside the first region).
namespace {

bool ext_contained(const bsw_params_t &p, int a, const bsw_ext_opt_t &opt, const bsw_seed_t &s, int l_query,
                   const bsw_alnreg_t *out, const int32_t *av, int32_t nav)
{
    for (int32_t k = 0; k < nav; ++k) {
        const bsw_alnreg_t &q = out[av[k]];
        if (s.rbeg < q.rb || s.rbeg + s.len > q.re || s.qbeg < q.qb || s.qbeg + s.len > q.qe) continue;
        if (s.len - q.seedlen0 > .1 * l_query) continue;
        int qd = s.qbeg - q.qb;
        int64_t rd = s.rbeg - q.rb;
        int max_gap = cal_max_gap(p, a, opt.w, qd < rd ? qd : (int)rd);
        int w = std::min(max_gap, q.w);
        if (qd - rd < w && rd - qd < w) return true;
        qd = q.qe - (s.qbeg + s.len);
        rd = q.re - (s.rbeg + s.len);
        max_gap = cal_max_gap(p, a, opt.w, qd < rd ? qd : (int)rd);
        w = std::min(max_gap, q.w);
        if (qd - rd < w && rd - qd < w) return true;
    }
    return false;
}

// extend(nj, job read offsets / lengths / seeds / windows, regions out) runs one round's extensions
template <class Extend>
int chain_rounds(bsw_ctx_t *ctx, const bsw_ext_opt_t *opt, int64_t ref_len, const int64_t *read_off,
                 const int32_t *read_len, int32_t n_reads, const bsw_seed_t *seeds, const int32_t *seed_read, const int32_t *seed_chain,
                 int32_t ns, bsw_alnreg_t *out, int32_t *extended, bsw_chain_stats_t *cs, Extend extend)
{
    bsw_params_t p;
    bsw::ctx_params(ctx, &p);
    const int a = p.mat[0];
    *cs = bsw_chain_stats_t{};
    auto tp = Clock::now();
    // read runs (seeds grouped by read)
    std::vector<int32_t> rstart;
    rstart.reserve((size_t)std::max(1, n_reads) + 1);
    for (int32_t k = 0; k < ns; ++k) {
        if (seed_read[k] < 0 || seed_read[k] >= n_reads || (k > 0 && seed_read[k] < seed_read[k - 1]))
            return BSW_E_INVAL;
        if (k == 0 || seed_read[k] != seed_read[k - 1]) rstart.push_back(k);
    }
    const int32_t nrun = (int32_t)rstart.size();
    rstart.push_back(ns);
    // processing order per read: chains in order, each chain's seeds by (score, index) desc;
    // order[] positions of a chain coincide with its seed-index range
    std::vector<int32_t> order((size_t)ns), chain_of((size_t)ns);
    std::vector<int64_t> cwin(2 * (size_t)ns);          // the chain's target window, per chain head
    parallel_for(nrun, [&](int32_t r0, int32_t r1) {
        for (int32_t r = r0; r < r1; ++r) {
            for (int32_t k = rstart[r]; k < rstart[r + 1]; ++k) { memset(&out[k], 0, sizeof(out[k])); extended[k] = 0; }
            for (int32_t c0 = rstart[r]; c0 < rstart[r + 1];) {
                int32_t c1 = c0;
                while (c1 < rstart[r + 1] && seed_chain[c1] == seed_chain[c0]) ++c1;
                for (int32_t i = c0; i < c1; ++i) { order[i] = i; chain_of[i] = c0; }
                chain_window(p, a, *opt, ref_len, read_len[seed_read[c0]], c1 - c0,
                             [&](int i) -> const bsw_seed_t & { return seeds[c0 + i]; }, &cwin[2 * (size_t)c0],
                             &cwin[2 * (size_t)c0 + 1]);
                std::sort(order.begin() + c0, order.begin() + c1, [&](int32_t x, int32_t y) {
                    const int64_t kx = (int64_t)seeds[x].len * a, ky = (int64_t)seeds[y].len * a;
                    return kx != ky ? kx > ky : x > y;
                });
                c0 = c1;
            }
        }
    });
    // per read: next position in order[], regions so far (flat: av[rstart[r] ..], nav[r])
    std::vector<int32_t> pos(rstart.begin(), rstart.end() - 1), av((size_t)ns), nav((size_t)nrun, 0);
    std::vector<int32_t> pick((size_t)nrun), jobs, job_run, jcnt;
    std::vector<int64_t> joff, jwin;
    std::vector<int32_t> jlen;
    std::vector<bsw_seed_t> jseed;
    std::vector<bsw_alnreg_t> jout;
    cs->prep_ms = ms_since(tp);
    for (;;) {
        auto tc = Clock::now();
        parallel_for(nrun, [&](int32_t b0, int32_t b1) {
            for (int32_t r = b0; r < b1; ++r) {
                pick[r] = -1;
                while (pos[r] < rstart[r + 1]) {
                    const int32_t si = order[pos[r]++];
                    const bsw_seed_t &s = seeds[si];
                    const int l_query = read_len[seed_read[si]];
                    if (s.len > 0 && ext_contained(p, a, *opt, s, l_query, out, av.data() + rstart[r], nav[r])) {
                        // overlapping extended seeds of the same chain processed earlier
                        bool keep = false;
                        const int32_t c0 = chain_of[si];
                        for (int32_t q = c0; q < pos[r] - 1 && !keep; ++q) {
                            const int32_t ti = order[q];
                            if (!extended[ti]) continue;
                            const bsw_seed_t &t = seeds[ti];
                            if (t.len < s.len * .95) continue;
                            if (s.qbeg <= t.qbeg && s.qbeg + s.len - t.qbeg >= s.len >> 2 &&
                                t.qbeg - s.qbeg != t.rbeg - s.rbeg) keep = true;
                            if (t.qbeg <= s.qbeg && t.qbeg + t.len - s.qbeg >= s.len >> 2 &&
                                s.qbeg - t.qbeg != s.rbeg - t.rbeg) keep = true;
                        }
                        if (!keep) continue;           // skipped, next seed of this read
                    }
                    pick[r] = si;
                    break;
                }
            }
        });
        jobs.clear(); job_run.clear();
        for (int32_t r = 0; r < nrun; ++r)
            if (pick[r] >= 0) { jobs.push_back(pick[r]); job_run.push_back(r); }
        cs->check_ms += ms_since(tc);
        if (jobs.empty()) break;
        const int32_t nj = (int32_t)jobs.size();
        joff.resize(nj); jlen.resize(nj); jseed.resize(nj); jout.resize(nj); jwin.resize(2 * (size_t)nj);
        parallel_for(nj, [&](int32_t k0, int32_t k1) {
            for (int32_t k = k0; k < k1; ++k) {
                const int32_t si = jobs[k], rid = seed_read[si];
                joff[k] = read_off[rid]; jlen[k] = read_len[rid]; jseed[k] = seeds[si];
                jwin[2 * k] = cwin[2 * (size_t)chain_of[si]];
                jwin[2 * k + 1] = cwin[2 * (size_t)chain_of[si] + 1];
            }
        });
        auto te = Clock::now();
        const int rc = extend(nj, joff.data(), jlen.data(), jseed.data(), jwin.data(), jout.data());
        if (rc) return rc;
        cs->ext_ms += ms_since(te);
        bsw_ext_stats_t es{};
        bsw::get_ext_stats(ctx, &es);
        for (int q = 0; q < 4; ++q) cs->n_pairs[q] += es.n_pairs[q];
        cs->kernel_ms += es.kernel_ms;
        parallel_for(nj, [&](int32_t k0, int32_t k1) {
            for (int32_t k = k0; k < k1; ++k) {
                const int32_t si = jobs[k], r = job_run[k];
                out[si] = jout[k];
                extended[si] = 1;
                av[rstart[r] + nav[r]++] = si;
            }
        });
        cs->rounds++;
        cs->n_extended += nj;
    }
    cs->n_skipped = ns - cs->n_extended;
    return BSW_OK;
}

}  // namespace

extern "C" int bsw_chain2aln(bsw_ctx_t *ctx, const bsw_ext_opt_t *opt, const uint8_t *ref, int64_t ref_len,
                             const uint8_t *reads, const int64_t *read_off, const int32_t *read_len, int32_t n_reads,
                             const bsw_seed_t *seeds, const int32_t *seed_read, const int32_t *seed_chain,
                             int32_t n_seeds, bsw_alnreg_t *out, int32_t *extended)
{
    if (!ctx || !opt || n_seeds < 0 || n_reads < 0 ||
        (n_seeds > 0 && (!ref || !reads || !read_off || !read_len || !seeds || !seed_read || !seed_chain || !out ||
                         !extended)))
        return BSW_E_INVAL;
    if (const int rc = bsw::ext_opt_check(opt, ref_len)) return rc;
    bsw_chain_stats_t cs{};
    const int rc = chain_rounds(ctx, opt, ref_len, read_off, read_len, n_reads, seeds, seed_read, seed_chain, n_seeds,
                                out, extended, &cs,
                                [&](int32_t nj, const int64_t *jo, const int32_t *jl, const bsw_seed_t *js,
                                    const int64_t *jw, bsw_alnreg_t *jr) {
                                    return extend_seeds_win(ctx, opt, ref, ref_len, reads, jo, jl, js, jw, nj, jr);
                                });
    bsw::set_chain_stats(ctx, cs);
    return rc;
}

// bsw_chain2aln_device / bsw_chain2aln_resident: csrc/bsw_chain.hip (GPU rounds)

extern "C" int bsw_chain_last_stats(bsw_ctx_t *ctx, bsw_chain_stats_t *out)
{
    return bsw::get_chain_stats(ctx, out);
}
