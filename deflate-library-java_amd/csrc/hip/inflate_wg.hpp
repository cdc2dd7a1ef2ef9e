// inflate_wg.hpp -- workgroup rounds: W waves decode one chain's rounds together (count pass).
//
// The one-wave count pass (ndfl_inflate_count_wave_kernel) decodes a block in rounds of 64 lane
// segments, one round after another; a block of ~270 Kbit takes ~10 rounds in sequence, so the
// decode needs a chain start (a header candidate) at nearly every block to keep the chip busy --
// which is what the dense header finder pays for.  Here a workgroup of W waves runs each round
// over 64W lane segments ("virtual lanes" L = 64 * wave + lane): the same speculative decode,
// verify and fix-up steps per lane (wv::spec_run / verify_run / phase_multi), with:
//   * one set of decode tables per workgroup (built by wave 0, shared in LDS);
//   * each wave staging its own 64 lanes' input (its own Stage);
//   * the verify of a wave's lane 0 starting from the previous wave's lane 63 speculative exit
//     (after a workgroup barrier), the fix-up sweeps wave-local (wave synchronisation only: their
//     trip counts differ between waves), and a final in-order pass over the waves that re-runs a
//     wave only when its predecessor's exit moved in its own sweeps (rare);
//   * phase-mapped rounds composing the phase maps across waves (per-wave scan, then the waves'
//     totals in order).
// A round's records go out per wave (64 lanes each, linked in order), so the emit pass replays
// them as it replays the one-wave kernel's: SegMeta::rs names each record's staging origin.
// Reference: the same decode as D/decomp/Open.java:446-618, one symbol at a time there.
#pragma once

namespace wv {

template <int W>
struct WgX {
    uint32_t exit_[64 * W];       // current exits (fix-up sweeps)
    uint32_t sx_[64 * W];         // speculative exits (written once per round, read across waves)
    uint8_t kind_[64 * W];
    uint64_t m[2][W];             // per-wave ballots / sums, double-buffered: one barrier per reduction
    uint32_t pe[W][8];            // phase-mapped rounds: lane 63's eight phase ends
    uint32_t qt[W];               // phase-mapped rounds: the wave's composed phase map
    uint32_t xs[W];               // phase-mapped rounds: lane 63's exit at its phase
    uint32_t ftw[W];              // first terminating lane of each wave (64: none)
    uint32_t nsl[W];              // unsynchronised lanes of each wave in the round
    uint64_t b64[4];              // broadcasts
    uint32_t b32[8];
};

template <int W>
__device__ __forceinline__ void wg_masks(bool p, WgX<W>& X, uint32_t& par, uint64_t (&M)[W]) {
    const uint64_t m = __ballot(p);
    if ((threadIdx.x & 63) == 0) X.m[par][threadIdx.x >> 6] = m;
    __syncthreads();
#pragma unroll
    for (int w = 0; w < W; w++) M[w] = X.m[par][w];
    par ^= 1;
}
// first virtual lane with p (64W: none); every thread of the workgroup calls
template <int W>
__device__ __forceinline__ uint32_t wg_first(bool p, WgX<W>& X, uint32_t& par) {
    uint64_t M[W];
    wg_masks<W>(p, X, par, M);
    uint32_t r = 64 * W;
#pragma unroll
    for (int w = W - 1; w >= 0; w--)
        if (M[w]) r = 64 * (uint32_t)w + (uint32_t)__builtin_ctzll(M[w]);
    return r;
}
template <int W>
__device__ __forceinline__ bool wg_all(bool p, WgX<W>& X, uint32_t& par) {
    return wg_first<W>(!p, X, par) == 64 * W;
}
template <int W>
__device__ __forceinline__ uint64_t wg_sum(uint64_t v, WgX<W>& X, uint32_t& par) {
    const uint64_t t = wave_sum_u64(v);
    if ((threadIdx.x & 63) == 0) X.m[par][threadIdx.x >> 6] = t;
    __syncthreads();
    uint64_t r = 0;
#pragma unroll
    for (int w = 0; w < W; w++) r += X.m[par][w];
    par ^= 1;
    return r;
}

// Round geometry over 64W lane segments (make_geo for one wave); MAX_SPAN_W caps a round.
template <int W>
__device__ __forceinline__ Geo make_geo_w(const In& in, uint64_t rs, uint64_t E) {
    Geo g;
    g.base = rs & ~31ull;
    g.r0 = (uint32_t)(rs - g.base);
    g.re = (uint32_t)(E - g.base);
    const uint32_t span = g.re - g.r0;
    g.pw = max((uint32_t)NDFL_PW_MIN, ((span + 64 * W - 1) / (64 * W) + 31) / 32);
    g.nb = (uint32_t)min(in.nbits - min(in.nbits, g.base), (uint64_t)0xFFFFFFFFu);
    return g;
}
template <int W>
__device__ __forceinline__ void lane_seg_w(const Geo& g, uint32_t L, uint32_t& s, uint32_t& e) {
    const uint32_t per = g.pw * 32;
    s = min(g.r0 + L * per, g.re);
    e = L == 64 * W - 1 ? g.re : min(g.r0 + (L + 1) * per, g.re);
}
// one wave stages its 64 lanes' regions (virtual lanes L = 64 * wave + lane)
__device__ __forceinline__ void stage_wave(const In& in, const Geo& g, Stage& st, uint32_t L) {
    const uint64_t w0 = (g.base >> 5) + (uint64_t)L * g.pw;
    const uint64_t wmax = in.nwords + 60;          // inside the IN_PAD zero bytes after the input
    const int lane = threadIdx.x & 63;
    wsync();                                       // this wave's reads of the previous round are done
#pragma unroll 4
    for (uint32_t i = 0; i < SW; i++)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(in.w + min(w0 + i, wmax)),
                                         (__attribute__((address_space(3))) void*)&st.w[i * 64], 4, 0, NDFL_STAGE_CPOL);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wsync();
    (void)lane;
}

// Phase runs 1..7 of the lanes after `from` (the fallback of round_decode), into the wave's slot.
__device__ __forceinline__ void phase_runs_w(const Lv& v, const Tabs& t, bool ed, uint32_t nb, uint32_t s, uint32_t e,
                                             uint32_t C1, PhArr* ph, int lane, uint32_t from, bool& phok) {
    if ((uint32_t)lane > from) {
        for (uint32_t f = 1; f < NPH; f++) {
            Spec q;
            spec_run(v, t, ed, nb, min(s + f, e), s, C1, C1, e, q);
            ph->cp[f - 1][lane] = (q.cp1 < 0xFFFFu && q.cpc1 <= 0xFFFFu) ? (q.cp1 | (q.cpc1 << 16)) : 0xFFFFu;
            ph->end[f - 1][lane] = q.end - s;
            ph->cnt[f - 1][lane] = q.cnt;
            ph->kr[f - 1][lane] = (uint8_t)((q.kind << 5) | q.reason);
        }
        phok = true;
    }
}

// Wave-local fix-up sweeps (round_decode's, wave synchronisation only): every lane whose start is
// not its predecessor's current exit re-runs its verify from that exit; lane 0's predecessor exit
// is `l0start`.  Returns the wave's first terminating lane (64: none).
template <int W>
__device__ __forceinline__ uint32_t wave_sweeps(const Lv& v, const Tabs& t, bool ed, uint32_t nb, uint32_t s, uint32_t e,
                                                uint32_t C1, uint32_t C2, const Spec& p0, PhArr* ph, WgX<W>& X,
                                                uint32_t l0start, uint32_t& nph, bool& phok, SegR& r, uint32_t& nfix) {
    const int lane = threadIdx.x & 63;
    const uint32_t L = threadIdx.x;
    uint32_t ftw = 64u;
    uint64_t chgm = 0;
    for (;;) {
        wsync();
        const uint32_t st = lane ? X.exit_[L - 1] : l0start;
        const bool inc = st != r.start;
        const uint64_t cm = __ballot(inc);
        const uint32_t fc = cm ? (uint32_t)__builtin_ctzll(cm) : 64u;
        const uint64_t tx = __ballot((uint32_t)lane < fc && r.kind != T_EXIT);
        if (tx) { ftw = (uint32_t)__builtin_ctzll(tx); break; }
        if (!cm) break;
        nfix++;
        const bool pchg = lane > 0 && ((chgm >> (lane - 1)) & 1ull);
        const bool redo = inc && ((uint32_t)lane == fc || !pchg);
        const uint32_t old_end = r.end;
        bool met = true;
        if (redo) met = verify_run(v, t, ed, nb, st, s, C1, C2, e, p0, ph, lane, phok ? nph : 1u, r);
        if (nph == 1 && __any((uint32_t)lane == fc && !met)) { phase_runs_w(v, t, ed, nb, s, e, C1, ph, lane, fc, phok); nph = NPH; }
        chgm = __ballot(redo && r.end != old_end);
        wsync();                                // every lane has read its predecessor's exit
        if (redo) X.exit_[L] = r.end;
    }
    return ftw;
}

// One round over [rs, E) on 64W lanes.  first_term: first virtual lane ending the block (64W: none);
// nsl: unsynchronised lanes of the round (all waves).  Every thread of the workgroup calls.
template <int W>
__device__ void round_decode_wg(const In& in, const Tabs& t, bool ed, uint64_t rs, uint64_t E, WgX<W>& X, Stage* stg,
                                Seg& out, uint32_t& first_term, uint32_t& nsl, uint32_t& nfix, PhArr* ph, Geo& g) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t L = threadIdx.x;
    g = make_geo_w<W>(in, rs, E);
    stage_wave(in, g, stg[wave], L);
    Lv v;
    v.p = stg[wave].w + lane;
    v.rw = L * g.pw;
    const uint32_t nb = g.nb;
    uint32_t s, e;
    lane_seg_w<W>(g, L, s, e);
    const uint32_t C1 = s + min(XCP1, e - s), C2 = s + min(XCP2, e - s);
    Spec p0;
    spec_run(v, t, ed, nb, s, s, C1, C2, e, p0);
    X.sx_[L] = p0.end;
    __syncthreads();
    SegR r;
    bool fin;
    if (L == 0) {
        r.start = s; r.end = p0.end; r.cnt = p0.cnt; r.kind = p0.kind; r.reason = p0.reason;
        fin = true;
    } else {
        fin = verify_run(v, t, ed, nb, X.sx_[L - 1], s, C1, C2, e, p0, ph, lane, 1, r);
    }
    // wave-local resolution; lane 0 of a wave takes its start as given (wave 0: the round start,
    // wave w > 0: wave w - 1's speculative exit, checked in order below)
    const uint64_t um = __ballot(!fin);
    const uint32_t j0 = um ? (uint32_t)__builtin_ctzll(um) : 64u;
    const uint64_t tm = __ballot(fin && r.kind != T_EXIT);
    const uint32_t t0 = tm ? (uint32_t)__builtin_ctzll(tm) : 64u;
    uint32_t nph = 1;
    bool phok = false;
    uint32_t ftw = t0;
    X.exit_[L] = r.end;
    if (j0 < t0) {
        nph = __popcll(um) > NDFL_PH_FALLBACK ? NPH : 1u;
        if (nph > 1) phase_runs_w(v, t, ed, nb, s, e, C1, ph, lane, j0, phok);
        // (lane 0's start stays as given here: its own r.start is passed as its predecessor's exit)
        ftw = wave_sweeps<W>(v, t, ed, nb, s, e, C1, C2, p0, ph, X, r.start, nph, phok, r, nfix);
    }
    if (lane == 0) { X.ftw[wave] = ftw; X.nsl[wave] = (j0 < t0) ? (uint32_t)__popcll(um) : 0u; }
    __syncthreads();
    // in order over the waves: wave w is exact when wave w - 1's final exit is the speculative one
    // its lane 0 verified from; otherwise it re-runs from the final exit (its sweeps take it on)
    for (int w = 1; w < W; w++) {
        if (X.ftw[w - 1] < 64u) break;                   // the block ended in an earlier wave
        const uint32_t fx = X.exit_[64 * w - 1];
        if (fx == X.sx_[64 * w - 1]) continue;           // (uniform: LDS after a barrier)
        if (wave == w) {
            // lane 0 re-verifies from the final exit; the sweeps carry the change on
            const uint32_t ft2 = wave_sweeps<W>(v, t, ed, nb, s, e, C1, C2, p0, ph, X, fx, nph, phok, r, nfix);
            if (lane == 0) X.ftw[wave] = ft2;
        }
        __syncthreads();
    }
    first_term = 64u * W;
    nsl = 0;
#pragma unroll
    for (int w = 0; w < W; w++) {
        nsl += X.nsl[w];
        if (first_term == 64u * W && X.ftw[w] < 64u) first_term = 64u * (uint32_t)w + X.ftw[w];
    }
    out.start = g.base + r.start; out.end = g.base + r.end; out.cnt = r.cnt;
    out.kind = r.kind; out.reason = r.reason;
}

// Phase-mapped round over 64W lanes (round_decode_phased, the maps composed across the waves).
template <int W>
__device__ void round_decode_phased_wg(const In& in, const Tabs& t, bool ed, uint64_t rs, uint64_t E, WgX<W>& X,
                                       Stage* stg, Seg& out, uint32_t& first_term, uint32_t& nfix, Geo& g, uint32_t& par,
                                       uint32_t esc4) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t L = threadIdx.x;
    g = make_geo_w<W>(in, rs, E);
    stage_wave(in, g, stg[wave], L);
    Lv v;
    v.p = stg[wave].w + lane;
    v.rw = L * g.pw;
    const uint32_t nb = g.nb;
    uint32_t s, e;
    lane_seg_w<W>(g, L, s, e);
    uint32_t endv[8], cntv[8], fbcv[8], krv[8];
    uint32_t fbl = 0, fbh = 0;
    {
        PhOut P[8];
        if (esc4) phase_multi_esc<8>(v, t, ed, nb, s, e, esc4, P);
        else phase_multi<8>(v, t, ed, nb, s, e, P);    // (past e: empty, ends at s + f)
#pragma unroll
        for (uint32_t h = 0; h < 8; h++) {
            endv[h] = P[h].end; cntv[h] = P[h].cnt; fbcv[h] = P[h].fbc; krv[h] = P[h].kr;
            const uint32_t fo = (P[h].fb != NOCP && P[h].fb - s < 255u) ? P[h].fb - s : 255u;
            if (h < 4) fbl |= fo << (8 * h); else fbh |= fo << (8 * (h - 4));
        }
    }
    if (lane == 63) {
#pragma unroll
        for (uint32_t f = 0; f < 8; f++) X.pe[wave][f] = endv[f];
    }
    __syncthreads();
    // map of lane L: phase of lane L - 1 -> phase of lane L (lane 0 of the round: always phase 0)
    uint32_t Q = 0;
#pragma unroll
    for (uint32_t f = 0; f < 8; f++) {
        uint32_t x = __shfl_up(endv[f], 1, 64);
        if (lane == 0) x = wave > 0 ? X.pe[wave - 1][f] : 0u;
        const uint32_t vv = phase_of(x - s, fbl, fbh) & 15u;
        if (L > 0) Q |= vv << (4 * f);
    }
#pragma unroll
    for (int k = 1; k < 64; k <<= 1) {
        const uint32_t B = __shfl_up(Q, k, 64);
        if (lane >= k) Q = map_compose(Q, B);
    }
    if (lane == 63) X.qt[wave] = Q;
    __syncthreads();
    if (wave > 0) {
        uint32_t P = X.qt[0];
        for (int w = 1; w < wave; w++) P = map_compose(X.qt[w], P);
        Q = map_compose(Q, P);
    }
    const uint32_t myph = Q & 15u;
    const uint32_t xsel = myph < 8 ? sel8(endv, myph) : NOCP;
    if (lane == 63) X.xs[wave] = xsel;
    __syncthreads();
    uint32_t x = __shfl_up(xsel, 1, 64);
    if (lane == 0) x = wave > 0 ? X.xs[wave - 1] : s;
    SegR r;
    r.start = x; r.end = x; r.cnt = 0; r.kind = T_ERR; r.reason = R_INTERNAL;
    bool known = false;
    if (myph < 8) {
        const uint32_t pc = phase_of(x - s, fbl, fbh);
        const uint32_t f = pc & 15u;
        if (f == myph) {
            known = true;
            const uint32_t kr = sel8(krv, f);
            r.end = sel8(endv, f);
            r.cnt = sel8(cntv, f) - ((pc & 16u) ? sel8(fbcv, f) : 0u);
            r.kind = kr >> 5; r.reason = kr & 31u;
        }
    }
    const uint32_t u = wg_first<W>(!known, X, par);
    const uint32_t t0 = wg_first<W>(known && r.kind != T_EXIT, X, par);
    first_term = t0;
    if (u < t0) {
        // in-order decode from lane u on (its predecessor is exact)
        X.exit_[L] = r.end;
        __syncthreads();
        first_term = 64u * W;
        for (uint32_t j = u; j < 64u * W && first_term == 64u * W; j++) {
            nfix++;
            if (L == j) {
                const uint32_t st = j ? X.exit_[j - 1] : s;
                uint32_t en, cn, kr, fb, fbc;
                if (esc4) {
                    PhOut P1[1];
                    phase_multi_esc<1>(v, t, ed, nb, st, e, esc4, P1);
                    en = P1[0].end; cn = P1[0].cnt; kr = P1[0].kr;
                } else {
                    phase_run(v, t, ed, nb, st, e, en, cn, kr, fb, fbc);
                }
                r.start = st; r.end = en; r.cnt = cn; r.kind = kr >> 5; r.reason = kr & 31u;
                X.exit_[L] = en;
                X.kind_[L] = (uint8_t)r.kind;
            }
            __syncthreads();
            if (X.kind_[j] != T_EXIT) first_term = j;
        }
    }
    out.start = g.base + r.start; out.end = g.base + r.end; out.cnt = r.cnt;
    out.kind = r.kind; out.reason = r.reason;
}

}  // namespace wv

// Count pass, W waves per chain (see the top of this file).  Arguments as
// ndfl_inflate_count_wave_kernel; ph_all holds one phase-fallback slot per wave of the grid.
template <int W>
__global__ void __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(NDFL_COUNT_WPE)))
ndfl_inflate_count_wg_kernel(const uint32_t* w, uint64_t nwords, uint64_t nbits, const uint64_t* starts,
                             const uint64_t* stops, uint32_t nchains, const uint64_t* cands, uint32_t ncand,
                             uint64_t limit, ChainRes* res, uint32_t* stats, uint64_t slot_base, SegPool pool,
                             uint32_t* ticket, wv::PhArr* ph_all, const uint32_t* order, uint64_t stop_all,
                             const wv::HdrRec* hrec, const uint32_t* nord, const uint32_t*, const uint32_t*) {
    using namespace wv;
    __shared__ __attribute__((aligned(16))) Shared S;
    if (nord) nchains = *nord;                  // (stored-header aliases left out of the order)
    __shared__ __attribute__((aligned(16))) WgX<W> X;
    __shared__ Stage stg[W];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t L = (uint32_t)tid;
    constexpr uint32_t NL = 64 * W;
    constexpr uint64_t SPAN_W = RSPAN * W;
    PhArr* ph = ph_all + (uint64_t)blockIdx.x * W + wave;
    const In in{w, nwords, nbits};
    uint32_t par = 0;
    // round and table records claimed in batches (thread 0's counters; the indices are broadcast)
    uint32_t rb_next = 0, rb_end = 0, tb_next = 0, tb_end = 0;
    for (;;) {
    __syncthreads();
    if (tid == 0) X.b32[0] = atomicAdd(ticket, 1u);
    __syncthreads();
    const uint32_t tk = X.b32[0];
    if (tk >= nchains) break;
    const uint32_t c = order[tk];
    const uint64_t start = starts[c], stop = stops ? stops[c] : stop_all;
    uint64_t cur = start, total = 0, endpos = start;
    uint32_t status = ST_BOUNDARY, reason = 0, nslow = 0, nfix = 0, nround = 0, next_idx = 0xFFFFFFFFu;
    bool recording = slot_base + c < pool.nslot;
    uint32_t prev_rec = NOREC;
    CandCur cc;
    if (slot_base == 0 && c < ncand) {
        cc.c = cands; cc.n = ncand; cc.i = c; cc.v = cands[c];
    } else {
        cc.init(cands, ncand, start);
    }
    for (int blk = 0;; blk++) {
        if (blk > 0 && (cur >= stop || cc.at(cur, &next_idx))) { status = ST_BOUNDARY; endpos = cur; break; }
        __syncthreads();                            // the previous block's table reads are done
        if (hrec && blk == 0 && cc.i < cc.n && cc.v == cur) {
            const HdrRec* hr = hrec + cc.i;
            uint32_t* lw = (uint32_t*)S.lens;
            if (tid < 80) lw[tid] = hr->lens[tid];
            if (tid == 0) hdr_to_shared(hr->h, S);
            __syncthreads();
        } else {
            for (uint32_t q = (uint32_t)tid; q < 320; q += NL) S.lens[q] = 0;
            __syncthreads();
            if (tid == 0) parse_hdr(in, cur, S);
            __syncthreads();
        }
        if (S.h_err) { status = ST_ERROR; reason = S.h_err; endpos = S.h_pos; break; }
        const uint64_t d0 = S.h_d0;
        const bool bfinal = S.h_bfinal != 0;
        if (S.h_btype == 0) {
            const uint64_t avail = (nbits - d0) / 8, ln = S.h_len;
            if (avail < ln) { total += avail; status = ST_ERROR; reason = R_UEOS; endpos = d0 + 8 * avail; break; }
            total += ln;
            cur = d0 + 8 * ln;
            if (bfinal) { status = ST_FINAL; endpos = cur; break; }
            continue;
        }
        // wave 0 builds the block's tables alone (wave synchronisation), the others wait
        if (wave == 0) {
            bool ed0;
            const int te0 = build_tables<true>(S, lane, ed0, stg[0].w);
            if (lane == 0) { X.b32[1] = (uint32_t)te0; X.b32[2] = ed0 ? 1u : 0u; }
        }
        __syncthreads();
        const int te = (int)X.b32[1];
        const bool ed = X.b32[2] != 0;
        if (te) { status = ST_ERROR; reason = (uint32_t)te; endpos = d0; break; }
        bool phased;
        {
            uint32_t n8 = 0;                        // (every wave counts the same lengths)
            for (uint32_t q = 0; q < 5; q++) {
                const uint32_t sy = q * 64 + (uint32_t)lane;
                n8 += (uint32_t)__popcll(__ballot(sy < 288 && S.lens[sy] == 8));
            }
            phased = n8 >= 192;
        }
        const uint32_t esc4 = (phased && NDFL_PHASE_ESC) ? flat8_mask(S.t, lane) : 0u;
        uint32_t brec = NOREC;
        if (recording && pool.nbt) {
            if (tid == 0) {
                if (tb_next >= tb_end) {
                    const uint32_t b = atomicAdd(pool.bctr, (uint32_t)NDFL_TREC_BATCH);
                    tb_next = b; tb_end = b + NDFL_TREC_BATCH;
                }
                X.b32[3] = tb_next++;
            }
            __syncthreads();
            brec = X.b32[3];
            if (brec < pool.nbt) {
                uint4* dst = (uint4*)(pool.bt + (uint64_t)brec * BT_BYTES);
                const uint4* src = (const uint4*)&S.t;
                for (uint32_t q = (uint32_t)tid; q < sizeof(Tabs) / 16; q += NL) dst[q] = src[q];
                if (tid == 0) {
                    uint64_t* h = (uint64_t*)(pool.bt + (uint64_t)brec * BT_BYTES + sizeof(Tabs));
                    h[0] = cur; h[1] = d0;
                    uint32_t* h32 = (uint32_t*)(h + 2);
                    h32[0] = S.h_bfinal; h32[1] = S.h_btype; h32[2] = ed ? 1u : 0u;
                    h32[3] = phased ? (esc4 ? esc4 : 1u) : 0u;
                }
            } else {
                brec = NOREC;
            }
        }
        uint64_t rs = d0;
        bool block_done = false, chain_done = false;
        while (!block_done) {
            uint64_t E = min(cc.after(rs, limit), rs + SPAN_W);
            if (E <= rs) E = rs + 1;
            Seg r;
            uint32_t ft;
            Geo g;
            if (phased) {
                round_decode_phased_wg<W>(in, S.t, ed, rs, E, X, stg, r, ft, nfix, g, par, esc4);
            } else {
                uint32_t nsl = 0;
                round_decode_wg<W>(in, S.t, ed, rs, E, X, stg, r, ft, nsl, nfix, ph, g);
                nslow += nsl;
                if (nsl > (uint32_t)NDFL_PHASE_SWITCH * W) phased = true;   // phase-locked code: map the next rounds
            }
            const bool live = L <= ft;
            if (recording) {
                // one record per wave with live lanes, linked in order; SegMeta::rs = the wave's
                // staging origin (its lane 0's segment start)
                const uint32_t nlive = ft < NL ? ft / 64 + 1 : (uint32_t)W;
                const bool fits = wg_all<W>(!live || r.cnt < 0xFFFFFFFFull, X, par);
                if (fits && tid == 0) {
                    if (rb_next + nlive > rb_end) {
                        const uint32_t want = max((uint32_t)NDFL_REC_BATCH, nlive);
                        const uint32_t b = atomicAdd(pool.ctr, want);
                        rb_next = b; rb_end = b + want;
                    }
                    X.b32[4] = rb_next;
                    rb_next += nlive;
                }
                __syncthreads();
                const uint32_t idx0 = fits ? X.b32[4] : NOREC;
                if (fits && idx0 + nlive <= pool.nrec) {
                    if ((uint32_t)wave < nlive) {
                        const uint32_t idx = idx0 + (uint32_t)wave;
                        pool.start[(uint64_t)idx * 64 + lane] = r.start;
                        pool.cnt[(uint64_t)idx * 64 + lane] = (uint32_t)r.cnt;
                        const uint32_t wft = (ft >= 64u * (uint32_t)wave && ft < 64u * (uint32_t)wave + 64u) ? ft - 64u * (uint32_t)wave : 64u;
                        const int src = wft < 64 ? (int)wft : 63;
                        const uint64_t fe = __shfl((unsigned long long)r.end, src, 64);
                        const uint32_t fk = __shfl(r.kind, src, 64), fr = __shfl(r.reason, src, 64);
                        const uint64_t x63 = __shfl((unsigned long long)r.end, 63, 64);
                        uint32_t s0, e0;
                        lane_seg_w<W>(g, 64u * (uint32_t)wave, s0, e0);
                        if (lane == 0) {
                            SegMeta m;
                            m.ft = wft; m.kind_ft = fk; m.reason_ft = fr;
                            m.next = (uint32_t)wave + 1 < nlive ? idx + 1 : NOREC;
                            m.end_ft = fe; m.exit63 = x63; m.pw = g.pw;
                            m.pad = wave == 0 ? brec : NOREC;
                            m.rs = g.base + s0;
                            pool.meta[idx] = m;
                        }
                    }
                    if (tid == 0) {
                        if (prev_rec == NOREC) pool.head[slot_base + c] = idx0;
                        else pool.meta[prev_rec].next = idx0;
                    }
                    prev_rec = idx0 + nlive - 1;
                    brec = NOREC;
                } else {
                    recording = false;              // the emit pass re-derives the remaining rounds
                }
            }
            nround++;
            total += wg_sum<W>(live ? r.cnt : 0ull, X, par);
            if (ft < NL) {
                if (L == ft) { X.b64[0] = r.end; X.b32[5] = r.kind; X.b32[6] = r.reason; }
                __syncthreads();
                const uint64_t fe = X.b64[0];
                const uint32_t fk = X.b32[5], fr = X.b32[6];
                block_done = true;
                if (fk == T_ERR) { status = ST_ERROR; reason = fr; endpos = fe; chain_done = true; }
                else {
                    cur = fe;
                    if (bfinal) { status = ST_FINAL; endpos = cur; chain_done = true; }
                }
            } else {
                if (L == NL - 1) X.b64[1] = r.end;
                __syncthreads();
                rs = X.b64[1];
            }
        }
        if (chain_done) break;
    }
    if (tid == 0) {
        ChainRes o;
        o.end_bit = endpos; o.out_count = total; o.status = status; o.reason = reason;
        o.next = next_idx;
        o.pad = 0;
        o.bnd_bit = 0; o.bnd_cnt = 0;
        res[c] = o;
        if (stats) { atomicAdd(&stats[0], nslow); atomicAdd(&stats[1], nfix); atomicAdd(&stats[2], nround); }
    }
    }
}
