// A diagonal role for the ticketed Cholesky, round 4 -- LAB ONLY (tools/diag2_lab.hip includes it
// after ipm_blas.hip).  Measured: 63.7 K vs 67.3 K cycles for the round-3 role alone, no change
// inside k_potrf_block, and its instantiation there raised the SGPR spills 80 -> 700+, so the
// library does not include it.
//
// One workgroup (4 waves) factors the 128 x 128 diagonal block of a panel held in LDS as 36 packed
// 16 x 16 blocks, one 16-column block column J = 0..7 at a time (NewtonSolver.py:303-313's
// cho_factor, the latency-bound part of the factorization).  Per step J:
//
//   A. leaves: the sweep of the 16 x 16 diagonal block (J, J) -- the pivot chain, ~95 cycles per
//      column -- also solves every tile below it in the same pass (X = B L_JJ^-T, B = the tile's
//      rows) and, on identity rows, the inverse (X = I L_JJ^-T = L_JJ^-T).  Each leaf wave keeps a
//      copy of the diagonal rows in all four 16-lane groups (the DPP row broadcast reads the
//      multiplier L[c2][c] from its own group) and one target row set per group:
//        wave 0: tiles J+1 .. J+4          wave 1: identity (-> L_JJ^-T), tiles J+5 .. J+7
//      so after ONE sweep the whole block column J is final, L_JJ^-1 included.
//      Waves 2-3 meanwhile (off the chain): apply terms 0 .. J-1 to block column J+1 (left-looking
//      look-ahead), and publish block column J-1 for the row workgroups (packed L blocks, L^-1, the
//      write-back to A, then the progress word).
//   B. term J on block column J+1 (one 4-MFMA tile update per tile, spread over the four waves).
//
// Two barriers per step; nothing global on the chain (the round-3 role published from the leaf
// waves and waited for those stores before its barrier, and formed L^-1 by a separate 16-step
// substitution on wave 3).  Same results contract as diag_role<true, V> for full panels (nb == 128):
// L11 written back to A, pubL (packed blocks) and Dinv_J = L_JJ^-1 (column-major) stored with sc1,
// *progress >= J + 1 once block row J and Dinv_J are visible, LAPACK info on a non-positive pivot.
#pragma once

struct Diag2Smem {
  double sD[36 * 256];   // L11 as packed lower 16 x 16 blocks (column-major within a block)
  double sLT[2][256];    // L_JJ^-T of the last two steps (column-major), double-buffered
  int fail;
};

#ifdef IPM_STAMPS2
__device__ unsigned long long ipm_stamps2[4][8][8];   // [wave][J][phase]
#define ST2(J, k) do { if (lane == 0) ipm_stamps2[wv][(J)][(k)] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define ST2(J, k) do {} while (0)
#endif

// nb <= 128 columns (the last panel of a factorization may be partial: identity padding beyond nb,
// the steps stop after block column (nb - 1) / 16)
// V (lab variants; the library uses the default): bit 0 -- ONE leaf wave (wave 0: identity + tiles
// J+1 .. J+3 in its sweep); the tiles below J+3 are solved by MFMA with L_JJ^-1 in step B, and their
// term J is applied during the next step's A; publishing split over waves 2 (write-back) and 3
template <bool FUSED = true, int V = 0>
__device__ __forceinline__ void diag_role2(int64_t k0, int nb, double* __restrict__ A, int64_t lda,
                                           double* __restrict__ dinv_out, int* __restrict__ info, double* pubL,
                                           unsigned* progress, Diag2Smem& sm, unsigned* failw = nullptr) {
  double* sD = sm.sD;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;   // 4 waves
  const int fr = lane & 15, fk = lane >> 4;
  const int rr = lane & 15, g = lane >> 4;
  if (FUSED) __builtin_amdgcn_s_setprio(3);   // the chain's CU-mates are trailing-update tiles
  if (tid == 0) sm.fail = 0;
  const int nJ = (nb + 15) >> 4;
  const bool full = nb == 128 && ((lda & 1) == 0) && ((k0 & 1) == 0);
  // ---- the 36 lower blocks global -> LDS (global_load_lds_dwordx4, 1 KB per wave instruction)
  if (full) {
    int cnt = 0;
#pragma unroll
    for (int I = 0; I < 8; ++I)
#pragma unroll
      for (int J = 0; J <= I; ++J)
#pragma unroll
        for (int h = 0; h < 2; ++h, ++cnt)
          if ((cnt & 3) == wv) {
            const double* src = A + (k0 + J * 16 + (lane >> 3) + 8 * h) * lda + k0 + I * 16 + 2 * (lane & 7);
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                             (__attribute__((address_space(3))) void*)&sD[bidx(I, J) * 256 + h * 128],
                                             16, 0, FUSED ? 16 : 0);   // aux 16 = sc1
          }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    // partial panel / odd leading dimension: element loads, identity beyond nb
    for (int e = tid; e < 36 * 256; e += 256) {
      const int blk = e >> 8, w = e & 255, c = w >> 4, r = w & 15;
      int I = 0;
      while ((I + 1) * (I + 2) / 2 <= blk) ++I;
      const int J = blk - I * (I + 1) / 2;
      const int i = I * 16 + r, j = J * 16 + c;
      double v;
      if (i < nb && j < nb) v = (i >= j) ? (FUSED ? ld_sc1(A + (k0 + j) * lda + k0 + i) : A[(k0 + j) * lda + k0 + i]) : 0.0;
      else v = (i == j) ? 1.0 : 0.0;
      sD[e] = v;
    }
  }
  __syncthreads();

  // T_IK -= L_IP L_KP^T on one 16 x 16 tile (transposed MFMA layout, see diag_role)
  auto tile_update = [&](int I, int K, int P) {
    const int o = fk * 16 + fr, cb = bidx(I, K) * 256 + o;
    const int ab = bidx(K, P) * 256 + o, bb = bidx(I, P) * 256 + o;
    dbl4 acc;
    double av[4], bv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[r] = sD[cb + 64 * r];
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      av[s4] = -sD[ab + 64 * s4];
      bv[s4] = sD[bb + 64 * s4];
    }
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s4], bv[s4], acc, 0, 0, 0);
#pragma unroll
    for (int r = 0; r < 4; ++r) sD[cb + 64 * r] = acc[r];
  };
  // T_IK -= sum_{P < np} L_IP L_KP^T (two accumulators; the loads of term P+1 issued before the
  // MFMAs of term P)
  auto tile_update_n = [&](int I, int K, int np) {
    const int o = fk * 16 + fr, cb = bidx(I, K) * 256 + o;
    dbl4 x0, x1 = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int r = 0; r < 4; ++r) x0[r] = sD[cb + 64 * r];
    double av[4], bv[4];
    auto ld = [&](int P) {
      const int ab = bidx(K, P) * 256 + o, bb = bidx(I, P) * 256 + o;
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        av[s4] = -sD[ab + 64 * s4];
        bv[s4] = sD[bb + 64 * s4];
      }
    };
    ld(0);
    for (int P = 0; P < np; ++P) {
      double a2[4], b2[4];
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        a2[s4] = av[s4];
        b2[s4] = bv[s4];
      }
      if (P + 1 < np) ld(P + 1);
      x0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a2[0], b2[0], x0, 0, 0, 0);
      x1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a2[1], b2[1], x1, 0, 0, 0);
      x0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a2[2], b2[2], x0, 0, 0, 0);
      x1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a2[3], b2[3], x1, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) sD[cb + 64 * r] = x0[r] + x1[r];
  };
  // block column Jc of L11 -> A (lower part of the diagonal tile), and the packed blocks + the
  // inverse L_JcJc^-1 (column-major; element (r, c) = L^-T (c, r) = sLT[r * 16 + c]) -> the row
  // workgroups; one wave
  auto publish = [&](int Jc) {
    const double* lt = sm.sLT[Jc & 1];
    const int r2 = 2 * (lane & 7), c0 = lane >> 3;
    for (int I = Jc; I < 8; ++I) {
      const int cb = bidx(I, Jc) * 256;
      if (pubL) {
#pragma unroll
        for (int q = 0; q < 4; ++q) st_sc1(&pubL[cb + q * 64 + lane], sD[cb + q * 64 + lane]);
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int c = c0 + 8 * h, i = I * 16 + r2, j = Jc * 16 + c;
        const double2 v = *reinterpret_cast<const double2*>(&sD[cb + c * 16 + r2]);
        double* dst = A + (k0 + j) * lda + k0 + i;
        if (full && I > Jc) {
          *reinterpret_cast<double2*>(dst) = v;
        } else if (j < nb) {
          if (i < nb && (I > Jc || r2 >= c)) dst[0] = v.x;
          if (i + 1 < nb && (I > Jc || r2 + 1 >= c)) dst[1] = v.y;
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = q * 64 + lane, c = e >> 4, r = e & 15;   // Dinv (r, c) at c * 16 + r
      const double v = lt[r * 16 + c];
      if (pubL) st_sc1(&dinv_out[Jc * 256 + e], v);
      else dinv_out[Jc * 256 + e] = v;
    }
  };
  // X_IJ = A_IJ L_JJ^-T in place (MFMA; L_JJ^-T column-major in sLT: the A operand L^-1 (j, k) =
  // sLT[j * 16 + k])
  auto tile_solve = [&](int I, int J) {
    const int o = fk * 16 + fr, cb = bidx(I, J) * 256 + o;
    const double* lt = sm.sLT[J & 1];
    double av[4], bv[4];
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      av[s4] = lt[fr * 16 + fk + 4 * s4];
      bv[s4] = sD[cb + 64 * s4];
    }
    dbl4 acc = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s4], bv[s4], acc, 0, 0, 0);
#pragma unroll
    for (int r = 0; r < 4; ++r) sD[cb + 64 * r] = acc[r];
  };
  // publishing split over two waves (V & 1): part 0 the packed blocks + L^-1, part 1 the write-back
  auto publish_part = [&](int Jc, int part) {
    const double* lt = sm.sLT[Jc & 1];
    const int r2 = 2 * (lane & 7), c0 = lane >> 3;
    if (part == 0) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int e = q * 64 + lane, c = e >> 4, r = e & 15;
        const double v = lt[r * 16 + c];
        if (pubL) st_sc1(&dinv_out[Jc * 256 + e], v);
        else dinv_out[Jc * 256 + e] = v;
      }
      if (pubL) {
        for (int I = Jc; I < 8; ++I) {
          const int cb = bidx(I, Jc) * 256;
          double v[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] = sD[cb + q * 64 + lane];
#pragma unroll
          for (int q = 0; q < 4; ++q) st_sc1(&pubL[cb + q * 64 + lane], v[q]);
        }
      }
      return;
    }
    for (int I = Jc; I < 8; ++I) {
      const int cb = bidx(I, Jc) * 256;
      double2 v[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) v[h] = *reinterpret_cast<const double2*>(&sD[cb + (c0 + 8 * h) * 16 + r2]);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int c = c0 + 8 * h, i = I * 16 + r2, j = Jc * 16 + c;
        double* dst = A + (k0 + j) * lda + k0 + i;
        if (full && I > Jc) {
          *reinterpret_cast<double2*>(dst) = v[h];
        } else if (j < nb) {
          if (i < nb && (I > Jc || r2 >= c)) dst[0] = v[h].x;
          if (i + 1 < nb && (I > Jc || r2 + 1 >= c)) dst[1] = v[h].y;
        }
      }
    }
  };
  int bad = 0;
  if (V & 1) {
    // ======================================================================= one leaf wave
    for (int J = 0; J < nJ; ++J) {
      ST2(J, 0);
      if (wv == 0) {
        // ---- A: the leaf -- diagonal rows in every group, targets: g0 identity (-> L^-T), g1..3
        //      tiles J+1 .. J+3
        const int It = J + g;
        const bool ident = g == 0;
        const bool tval = !ident && It < nJ;
        const int db = bidx(J, J) * 256;
        const int src = tval ? bidx(It, J) * 256 : db;
        double row[16], rowb[16];
#pragma unroll
        for (int c = 0; c < 16; ++c) {
          row[c] = sD[db + c * 16 + rr];
          rowb[c] = ident ? (c == rr ? 1.0 : 0.0) : sD[src + c * 16 + rr];
        }
        double piv = readlane_d(row[0], 0);
        double dv = rsqrt_pivot(piv);
        int badl = 0;
#pragma unroll
        for (int c = 0; c < 16; ++c) {
          if (!(piv > 0.0) && badl == 0) badl = c + 1;
          double pivn = 1.0, dvn = 1.0;
          if (c + 1 < 16) {
            const double a1 = readlane_d(row[c], c + 1);
            const double d1 = readlane_d(row[c + 1], c + 1);
            const double l1 = a1 * dv;
            pivn = fma(-l1, l1, d1);
            dvn = rsqrt_pivot(pivn);
          }
          row[c] *= dv;
          rowb[c] *= dv;
#pragma unroll
          for (int c2 = c + 1; c2 < 16; ++c2) {
            fmac_bcast16(row[c2], row[c], row[c], c2, c2 == c + 1);
            fmac_bcast16(rowb[c2], row[c], rowb[c], c2, false);
          }
          piv = pivn;
          dv = dvn;
        }
#ifdef IPM_STAMPS2
        if (__builtin_amdgcn_readfirstlane(__double2hiint(rowb[15] + row[15])) == 0x7FF12345) sm.fail = -1;
#endif
        ST2(J, 1);
        if (tval) {
#pragma unroll
          for (int c = 0; c < 16; ++c) sD[src + c * 16 + rr] = rowb[c];
        } else if (ident) {
#pragma unroll
          for (int c = 0; c < 16; ++c) {
            sm.sLT[J & 1][c * 16 + rr] = rowb[c];
            sD[db + c * 16 + rr] = (rr >= c) ? row[c] : 0.0;
          }
          if (lane == 0 && badl) sm.fail = J * 16 + badl;
        }
        ST2(J, 2);
      } else {
        // ---- A, waves 1-3: term J-1 on tiles J+4 .. 7 of column J (solved in B of step J-1),
        //      terms 0 .. J-1 on column J+1 (look-ahead), publishing of column J-1 -- list-scheduled
        //      by cost (units ~ one 4-MFMA tile term): pubL + L^-1 8 (wave 3), write-back 4 (wave 2)
        int load[4] = {0, 0, J > 0 ? 4 : 0, J > 0 ? 8 : 0};
        auto pick = [&](int cost) {
          int b = 1;
#pragma unroll
          for (int w = 2; w < 4; ++w)
            if (load[w] < load[b]) b = w;
          load[b] += cost;
          return b;
        };
        if (J > 0) {
          if (wv >= 2) publish_part(J - 1, wv == 3 ? 0 : 1);   // (stores first: they drain meanwhile)
          ST2(J, 1);
          for (int I = J + 4; I < nJ; ++I)
            if (pick(1) == wv) tile_update(I, J, J - 1);
          if (J + 1 < nJ)
            for (int I = J + 1; I < nJ; ++I)
              if (pick(J) == wv) tile_update_n(I, J + 1, J);
          if (pubL) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        ST2(J, 2);
      }
      __syncthreads();
      // block row J-1 and L^-1_{J-1} are stored (every wave drained its stores before the barrier)
      if (J > 0 && pubL && tid == 0)
        __hip_atomic_fetch_max(progress, (unsigned)J, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      ST2(J, 3);
      if (sm.fail) {
        bad = sm.fail;
        break;
      }
      // ---- B: solve tiles J+4 .. 7 of column J (MFMA with L_JJ^-1), term J on tiles J+1 .. J+4 of
      //      column J+1 (what the next leaf reads)
      if (J + 1 < nJ) {
        const int I2 = J + 1 + wv;                        // wave w: term J on tile (J+1+w, J+1)
        if (wv == 3 && I2 < nJ) tile_solve(I2, J);        // (wave 3's tile J+4 first needs its solve)
        if (I2 < nJ) tile_update(I2, J + 1, J);
        const int I1 = J + 5 + wv;                        // waves 0-2: the solves of tiles J+5 .. J+7
        if (wv < 3 && I1 < nJ) tile_solve(I1, J);
        __syncthreads();
      }
      ST2(J, 4);
    }
  } else
  for (int J = 0; J < nJ; ++J) {
    ST2(J, 0);
    // ---------------------------------------------------------------- A. leaves / look-ahead
    if (wv < 2) {
      // target rows of this lane group: wave 0 tiles J+1+g; wave 1 g = 0 identity, tiles J+4+g
      const int It = wv == 0 ? J + 1 + g : J + 4 + g;
      const bool ident = wv == 1 && g == 0;
      const bool tval = !ident && It < 8;
      const int db = bidx(J, J) * 256;
      const int src = tval ? bidx(It, J) * 256 : db;   // absent tiles: a harmless diagonal copy
      double row[16], rowb[16];
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        row[c] = sD[db + c * 16 + rr];
        rowb[c] = ident ? (c == rr ? 1.0 : 0.0) : sD[src + c * 16 + rr];
      }
      double piv = readlane_d(row[0], 0);
      double dv = rsqrt_pivot(piv);
      int badl = 0;
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        if (!(piv > 0.0) && badl == 0) badl = c + 1;
        double pivn = 1.0, dvn = 1.0;
        if (c + 1 < 16) {
          const double a1 = readlane_d(row[c], c + 1);
          const double d1 = readlane_d(row[c + 1], c + 1);
          const double l1 = a1 * dv;
          pivn = fma(-l1, l1, d1);
          dvn = rsqrt_pivot(pivn);
        }
        row[c] *= dv;    // lane c: piv * dv = L_cc; other lanes: L[r][c]
        rowb[c] *= dv;   // X[r][c] of the target rows
#pragma unroll
        for (int c2 = c + 1; c2 < 16; ++c2) {
          fmac_bcast16(row[c2], row[c], row[c], c2, c2 == c + 1);
          fmac_bcast16(rowb[c2], row[c], rowb[c], c2, false);
        }
        piv = pivn;
        dv = dvn;
      }
      ST2(J, 1);
      if (tval) {
#pragma unroll
        for (int c = 0; c < 16; ++c) sD[src + c * 16 + rr] = rowb[c];
      } else if (ident) {
#pragma unroll
        for (int c = 0; c < 16; ++c) sm.sLT[J & 1][c * 16 + rr] = rowb[c];   // L^-T (rr, c)
      }
      if (wv == 0 && g == 0) {
#pragma unroll
        for (int c = 0; c < 16; ++c) sD[db + c * 16 + rr] = (rr >= c) ? row[c] : 0.0;
        if (lane == 0 && badl) sm.fail = J * 16 + badl;
      }
      ST2(J, 2);
    } else {
      // wave 3 publishes block column J-1 (stores drained here, off the chain, then the progress
      // word: block row J-1 and Dinv_{J-1} are visible); waves 2-3 apply terms 0 .. J-1 to block
      // column J+1 (tiles J+1 .. 7; wave 3 takes every third, it also publishes)
      if (wv == 3 && J > 0) {
        publish(J - 1);
        ST2(J, 1);
      }
      if (J > 0 && J + 1 < nJ) {
        int t = 0;
        for (int I = J + 1; I < 8; ++I, ++t)
          if ((wv == 3) == (t % 3 == 2)) tile_update_n(I, J + 1, J);
      }
      if (wv == 3 && J > 0 && pubL) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) __hip_atomic_fetch_max(progress, (unsigned)J, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      ST2(J, 2);
    }
    __syncthreads();
    ST2(J, 3);
    if (sm.fail) {
      bad = sm.fail;
      break;
    }
    // ---------------------------------------------------------------- B. term J on column J+1
    if (J + 1 < nJ) {
      for (int I = J + 1 + wv; I < 8; I += 4) tile_update(I, J + 1, J);
      __syncthreads();
    }
    ST2(J, 4);
  }
  if (bad) {
    if (tid == 0) {
      atomicCAS(info, 0, (int)(k0 + bad));
      __threadfence();   // (info before the failure word: a waiter released by failw cannot report first)
      if (failw) atomicCAS(failw, 0u, (unsigned)(k0 + bad));
      if (pubL) {
        __threadfence();
        __hip_atomic_fetch_max(progress, 0xFFFFFFFFu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    return;
  }
  // the last block column: published by wave 3, then every block row is visible
  if (V & 1) {
    if (wv >= 2) publish_part(nJ - 1, wv == 3 ? 0 : 1);
    if (pubL) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) __hip_atomic_fetch_max(progress, 8u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  } else if (wv == 3) {
    publish(nJ - 1);
    if (pubL) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) __hip_atomic_fetch_max(progress, 8u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}
#undef ST2
