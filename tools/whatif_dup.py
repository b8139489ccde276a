#!/usr/bin/env python3
"""Marginal cost of a kernel in throughput mode, measured by duplication.

Builds variants of libyrwi (never the product: a patched copy of csrc/ in /tmp,
output gpurun_var/libyrwi_dup_<name>.so) in which ONE idempotent launch is issued
twice in a row -- the second launch rewrites what the first wrote, so results stay
right, and the bench's step-time delta against the product build is what that
kernel costs among the other lanes' kernels.  Run the variants on the GPU box with
tools/ab.sh (YRWI_LIB).  Only kernels that are idempotent on the C2 workload
(default profile, 2-term, no authority) are listed.
  python3 tools/whatif_dup.py [names...]"""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "yacy_search_server_amd", "csrc")

K = "yrwi_kernels.hip"
VARIANTS = {
    "compact": [(K, "  hipLaunchKernelGGL(kc, dim3((unsigned)((total_tiles + COMPACT_TILES - 1) / COMPACT_TILES)), dim3(256), 0, S(st),\n"
                    "                     d_jobs, d_tile_base, njobs, total_tiles, d_pairs, d_pair_uid, d_tile_src, d_tile_cnt, d_tile_off,\n"
                    "                     perm, (const int32_t*)bo.tile_job);\n", 2)],
    "probe": [(K, "    hipLaunchKernelGGL(kp, dim3((unsigned)probe_tiles), dim3(PROBE_TILE), 0, S(st), d_jobs, d_tile_base, d_pdesc,\n"
                  "                       merge_tiles, d_pairs, d_pair_uid, d_tile_src, d_tile_cnt, (const int2*)pperm, d_tile_lvl,\n"
                  "                       (const ProbeDesc*)d_prange);\n", 2)],
    "reduce": [(K, "    hipLaunchKernelGGL(k_reduce, dim3((unsigned)total_chunks), dim3(CHUNK_THREADS),\n"
                   "                       hp_any ? HPART_MAXS * sizeof(int32_t) : 0, S(st), d_q, d_chunk_q, d_chunks, d_shard);\n", 2)],
    "shardfin": [(K, "  hipLaunchKernelGGL(k_shard_fin, dim3((unsigned)nq), dim3(64), 0, S(st), d_q, d_chunk_base, d_chunks, d_shard);\n", 2)],
    "combine": [(K, "  hipLaunchKernelGGL(k_combine, dim3((unsigned)((nq + 63) / 64)), dim3(64), 0, S(st), d_q, nq, d_shards, world, d_norm);\n", 2)],
    "emit": [(K, "  hipLaunchKernelGGL(k_emit, dim3((unsigned)nq), dim3(256), 0, S(st), d_q, nq, d_final, d_final_cnt, kmax,\n"
                 "                     d_hits, d_nout, mode);\n", 2)],
    "copyin": [(K, "  hipLaunchKernelGGL(k_copy_in, dim3(blocks), dim3(256), 0, (hipStream_t)stream, c);\n", 2)],
    "qtabs": [(K, "  hipLaunchKernelGGL(k_qtabs, dim3((unsigned)nq), dim3(256), 0, S(st), d_q, d_norm, qt);\n", 2)],
}
TOPQ = ("    hipLaunchKernelGGL(k_topq<4096>, dim3((unsigned)ngroups), dim3(TOPQ_THREADS), 2 * 4096 * sizeof(uint64_t), S(st),\n"
        "                       d_gbase, d_gn, d_gk, d_in, d_in_cnt, in_stride, keff, d_out, d_out_cnt);\n")
VARIANTS["topq"] = [(K, TOPQ, 2)]


# variants that change code rather than duplicate a launch: (file, old, new) edits
H = "yrwi_host.cpp"
def _compact_lds(kb):  # k_compact with kb KiB of unused dynamic LDS: fewer resident workgroups per CU
    return [(K, "hipLaunchKernelGGL(kc, dim3((unsigned)((total_tiles + COMPACT_TILES - 1) / COMPACT_TILES)), dim3(256), 0, S(st),",
             "hipLaunchKernelGGL(kc, dim3((unsigned)((total_tiles + COMPACT_TILES - 1) / COMPACT_TILES)), dim3(256), %d, S(st)," % (kb * 1024))]


EDITS = {
    "clds26": _compact_lds(26),
    "clds32": _compact_lds(32),
    "clds40": _compact_lds(40),
    # k_emit into a device buffer, then DMA copies to the pinned destination
    "emitdma": [
        (H, "  uint8_t* land = nullptr;\n  {\n    void* hp = h_hits;",
            "  uint8_t* land = nullptr;\n  void* hp_dst = nullptr;\n  void* np_dst = nullptr;\n  {\n    void* hp = h_hits;"),
        (H, "    HIPCHK(ctx, hipHostGetDevicePointer(reinterpret_cast<void**>(&d_hits), hp, 0));\n"
            "    HIPCHK(ctx, hipHostGetDevicePointer(reinterpret_cast<void**>(&d_nout), np, 0));\n  }",
            "    hp_dst = hp;\n    np_dst = np;\n    d_hits = arena_alloc<yrwi_hit>(ctx, (int64_t)nq * kmax);\n"
            "    d_nout = arena_alloc<int32_t>(ctx, nq);\n    if (!d_hits || !d_nout) return ctx->fail(YRWI_E_NOMEM, \"arena\");\n  }"),
        (H, "  if (tm) { tm->ts = ctx->event(); hipEventRecord(tm->ts, ctx->stream); }\n  HIPCHK(ctx, lane_sync(ctx));\n  if (hD_land) {",
            "  HIPCHK(ctx, hipMemcpyAsync(hp_dst, d_hits, hb, hipMemcpyDeviceToHost, ctx->stream));\n"
            "  HIPCHK(ctx, hipMemcpyAsync(np_dst, d_nout, nb, hipMemcpyDeviceToHost, ctx->stream));\n"
            "  if (tm) { tm->ts = ctx->event(); hipEventRecord(tm->ts, ctx->stream); }\n  HIPCHK(ctx, lane_sync(ctx));\n  if (hD_land) {"),
    ],
}


# k_compact also accumulating k_reduce's order-independent summary of the records
# it writes (packed min / max, tf fractions, pmax, count) plus a wave prefix max of
# posintext per pass, reduced per wave into a sink: what fusing the normalisation
# summary into the compaction would add to k_compact (results unchanged)
_CS_HELP = (K, "template <bool CHAIN>\n__global__ __launch_bounds__(256) void k_compact(",
            "typedef unsigned short wi_u16x2 __attribute__((ext_vector_type(2)));\n"
            "__device__ __forceinline__ uint32_t wi_min16(uint32_t a, uint32_t b) { return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(wi_u16x2, a), __builtin_bit_cast(wi_u16x2, b))); }\n"
            "__device__ __forceinline__ uint32_t wi_max16(uint32_t a, uint32_t b) { return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(wi_u16x2, a), __builtin_bit_cast(wi_u16x2, b))); }\n"
            "__device__ uint32_t g_wi_sink[1024];\n"
            "template <bool CHAIN>\n__global__ __launch_bounds__(256) void k_compact(")
_CS_INIT = (K, "  const int32_t total = sPre[COMPACT_TILES];\n  for (int m0 = threadIdx.x; m0 < total; m0 += COMPACT_UNROLL * 256) {",
            "  const int32_t total = sPre[COMPACT_TILES];\n"
            "  constexpr int WNP = (NF + 1) / 2;\n  uint32_t wmn[WNP], wmx[WNP];\n"
            "  for (int j = 0; j < WNP; j++) { wmn[j] = 0xFFFFFFFFu; wmx[j] = 0u; }\n"
            "  int32_t wpmax = -1, wnval = 0, wtcn = -1, wtdn = 1, wtcx = -1, wtdx = 1, wlastp = -1;\n  uint32_t wacc = 0;\n"
            "  for (int m0 = threadIdx.x; m0 < total; m0 += COMPACT_UNROLL * 256) {")
_CS_ACC = (K, "      store_rec(X.ofeat, o, (CHAIN && X.ctw) ? A[u] : joined_rec(A[u], B[u].x, B[u].y, X.mode, X.now_ms));\n"
              "      stg(X.ouid + o, uid[u]);\n    }\n  }\n}\n",
              "      const Rec R = (CHAIN && X.ctw) ? A[u] : joined_rec(A[u], B[u].x, B[u].y, X.mode, X.now_ms);\n"
              "      store_rec(X.ofeat, o, R);\n      stg(X.ouid + o, uid[u]);\n"
              "      const Feat F = decode_rec(R);\n"
              "      for (int j = 0; j < WNP; j++) {\n"
              "        const uint32_t w = (uint32_t)F.f[2 * j] | (2 * j + 1 < NF ? (uint32_t)F.f[2 * j + 1] << 16 : 0u);\n"
              "        wmn[j] = wi_min16(wmn[j], w); wmx[j] = wi_max16(wmx[j], w);\n      }\n"
              "      const int32_t tc = F.f[F_HITCOUNT], td = F.f[F_WORDSINTEXT] + F.f[F_WORDSINTITLE] + 1;\n"
              "      if (wtcn < 0 || tc * wtdn < wtcn * td) { wtcn = tc; wtdn = td; }\n"
              "      if (wtcx < 0 || wtcx * td < tc * wtdx) { wtcx = tc; wtdx = td; }\n"
              "      wpmax = max(wpmax, F.p); wnval++; wlastp = F.p;\n"
              "    }\n"
              "    int32_t pm = wlastp;\n"
              "    for (int o2 = 1; o2 < 64; o2 <<= 1) { const int32_t y = __shfl_up(pm, o2, 64); if ((threadIdx.x & 63) >= o2) pm = max(pm, y); }\n"
              "    wacc += (uint32_t)(pm > wlastp);\n"
              "  }\n"
              "  uint32_t h = wacc ^ (uint32_t)wpmax ^ (uint32_t)wnval ^ (uint32_t)(wtcn * 7 + wtdn * 3 + wtcx * 5 + wtdx);\n"
              "  for (int j = 0; j < WNP; j++) h ^= wmn[j] * 31u + wmx[j];\n"
              "  for (int o2 = 32; o2 > 0; o2 >>= 1) h ^= (uint32_t)__shfl_xor((int)h, o2, 64);\n"
              "  if ((threadIdx.x & 63) == 0 && h == 0x12345678u) g_wi_sink[blockIdx.x & 1023] = h;\n"
              "}\n")
EDITS["csum"] = [_CS_HELP, _CS_INIT, _CS_ACC]

# k_compact_sum's layout without its summaries: every step through the one-wave-per-tile
# kernel, no pieces (k_reduce reads the containers as before; results unchanged)
EDITS["sumlayout"] = [
    (H, "        J.want_sum = last && P.excl.empty() && P.prof.coeff_authority <= 12 ? 1 : 0;",
        "        J.want_sum = 0;"),
    (H, "  bool sum = false;\n  for (const JoinQ& J : jobs) sum |= J.want_sum != 0;",
        "  bool sum = true;\n  for (const JoinQ& J : jobs) sum |= J.want_sum != 0;"),
]

# a chained fold's pieces at a lower survivor density per tile (SUM_MIN_PER_TILE)
def _sum_min(v):
    return [("yrwi_internal.h", "constexpr int SUM_MIN_PER_TILE = 64;", "constexpr int SUM_MIN_PER_TILE = %d;" % v)]


EDITS["summin0"] = _sum_min(0)
EDITS["summin16"] = _sum_min(16)

# chained folds with exclusions inside the chain through k_compact_sum too
EDITS["chainexcl"] = [("yrwi_host.cpp",
                       "J.want_sum = last && P.excl.empty() && !chain_excl && P.prof.coeff_authority <= 12 ? 1 : 0;",
                       "J.want_sum = last && P.excl.empty() && (chain_excl || !chain_excl) && P.prof.coeff_authority <= 12 ? 1 : 0;")]


# variants that only change a compile-time constant (make EXTRA=...)
FLAGS = {
    "bm512": "-DYRWI_BM_TILE=512",
    "bm256": "-DYRWI_BM_TILE=256",
    "cu1": "-DYRWI_COMPACT_UNROLL=1",
    "cu3": "-DYRWI_COMPACT_UNROLL=3",
    "cu4": "-DYRWI_COMPACT_UNROLL=4",
}


def build(name):
    tmp = f"/tmp/whatif_{name}"
    shutil.rmtree(tmp, ignore_errors=True)
    src = os.path.join(tmp, "pkg", "csrc")  # the tree's shape: csrc/../../include/yrwi.h
    shutil.copytree(CSRC, src)
    os.makedirs(os.path.join(tmp, "include"), exist_ok=True)
    shutil.copy(os.path.join(ROOT, "include", "yrwi.h"), os.path.join(tmp, "include"))
    for f, text, times in VARIANTS.get(name, []):
        p = os.path.join(src, f)
        s = open(p).read()
        assert s.count(text) == 1, (name, f, s.count(text))
        s = s.replace(text, "{\n" + text * times + "}\n")  # (a braced block: some sit under an if)
        open(p, "w").write(s)
    for f, old, new in EDITS.get(name, []):
        p = os.path.join(src, f)
        s = open(p).read()
        assert s.count(old) == 1, (name, f, old[:60], s.count(old))
        open(p, "w").write(s.replace(old, new))
    out = os.path.join(ROOT, "gpurun_var", f"libyrwi_dup_{name}.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    subprocess.check_call(["make", "-s", "-j8", "-C", src, f"OUT={out}", f"OBJ={tmp}/obj",
                           "EXTRA=" + FLAGS.get(name, ""), out])
    print("built", out)


if __name__ == "__main__":
    for n in sys.argv[1:] or list(VARIANTS) + list(EDITS) + list(FLAGS):
        build(n)
