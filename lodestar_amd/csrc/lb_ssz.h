// SSZ merkleization on the GPU: hash_tree_root of many independent chunk lists at once, the
// hashing behind the signing roots the reference computes before verification --
// getBlockSignatureSets (state-transition/src/signatureSets/index.ts:64-111) ->
// computeSigningRoot = SigningData.hashTreeRoot (src/util/signingRoot.ts:7-13) over
// BeaconBlock / AttestationData / ... roots.  The host
// (lodestar_amd/signing_roots.py) walks the container types and batches every tree of one
// dependency level into one launch; this file is the hashing.
//
// Tree t: chunks [chunk_off[t], chunk_off[t+1]) (32 bytes each), padded with zero chunks to 2^depth
// leaves (the type's limit), optionally mixed with its length (lists / bitlists).  One thread
// per tree folds its level in place (chunks are scratch); levels past the real chunks hash with
// the precomputed zero-subtree roots.
#pragma once
#include "lb_h2c.h"

// SHA-256 of a 64-byte message (two 32-byte nodes): the data block, then the constant padding
// block (0x80, zeros, bit length 512).  Chunks are big-endian byte strings.
LB_HD void sha256_node(uint32_t out[8], const uint32_t l[8], const uint32_t r[8]) {
  uint32_t h[8], blk[16];
  sha256_init(h);
  LB_UNROLL for (int i = 0; i < 8; i++) {
    blk[i] = l[i];
    blk[8 + i] = r[i];
  }
  sha256_compress(h, blk);
  LB_UNROLL for (int i = 0; i < 16; i++) blk[i] = 0;
  blk[0] = 0x80000000u;
  blk[15] = 512u;
  sha256_compress(h, blk);
  LB_UNROLL for (int i = 0; i < 8; i++) out[i] = h[i];
}

LB_HD void chunk_ld(uint32_t w[8], const uint8_t* p) {
  LB_UNROLL for (int i = 0; i < 8; i++)
    w[i] = ((uint32_t)p[4 * i] << 24) | ((uint32_t)p[4 * i + 1] << 16) | ((uint32_t)p[4 * i + 2] << 8) | p[4 * i + 3];
}
LB_HD void chunk_st(uint8_t* p, const uint32_t w[8]) {
  LB_UNROLL for (int i = 0; i < 8; i++) {
    p[4 * i] = (uint8_t)(w[i] >> 24);
    p[4 * i + 1] = (uint8_t)(w[i] >> 16);
    p[4 * i + 2] = (uint8_t)(w[i] >> 8);
    p[4 * i + 3] = (uint8_t)w[i];
  }
}

// zero-subtree roots: zh[0] = 0^32, zh[d+1] = H(zh[d] || zh[d]).  Computed on the device (the
// SHA-256 round constants live in device constant memory).
LB_HD void ssz_zero_hashes(uint8_t* zh, int n) {
  uint32_t z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  chunk_st(zh, z);
  for (int d = 1; d < n; d++) {
    uint32_t nz[8];
    sha256_node(nz, z, z);
    LB_UNROLL for (int i = 0; i < 8; i++) z[i] = nz[i];
    chunk_st(zh + 32 * d, z);
  }
}

#if LB_KG(2)
__global__ void __launch_bounds__(64) k_ssz_zero_hashes(uint8_t* __restrict__ zh) {
  if (threadIdx.x == 0) ssz_zero_hashes(zh, 64);
}
#endif  // LB_KG

#define LB_SSZ_NO_MIX 0xffffffffffffffffull

#if LB_KG(2)
__global__ void __launch_bounds__(LB_TPB) k_merkleize(uint32_t n, const uint32_t* __restrict__ chunk_off,
                                                      const uint32_t* __restrict__ depth,
                                                      const uint64_t* __restrict__ mix_len,
                                                      uint8_t* __restrict__ chunks, const uint8_t* __restrict__ zh,
                                                      uint8_t* __restrict__ roots) {
  const uint32_t t = lb_tid();
  if (t >= n) return;
  uint8_t* c = chunks + (size_t)32 * chunk_off[t];
  uint32_t len = chunk_off[t + 1] - chunk_off[t];
  const uint32_t dep = depth[t];
  uint32_t root[8];
  if (len == 0) {
    chunk_ld(root, zh + 32 * dep);
  } else {
    for (uint32_t d = 0; d < dep; d++) {
      const uint32_t half = (len + 1) / 2;
      for (uint32_t i = 0; i < half; i++) {
        uint32_t l[8], r[8], o[8];
        chunk_ld(l, c + 64 * i);
        if (2 * i + 1 < len) chunk_ld(r, c + 64 * i + 32);
        else chunk_ld(r, zh + 32 * d);
        sha256_node(o, l, r);
        chunk_st(c + 32 * i, o);
      }
      len = half;
    }
    chunk_ld(root, c);
  }
  const uint64_t ml = mix_len[t];
  if (ml != LB_SSZ_NO_MIX) {
    uint32_t lw[8] = {0, 0, 0, 0, 0, 0, 0, 0}, o[8];
    // uint256 little-endian length as a big-endian-loaded chunk
    uint8_t lb[32];
    for (int i = 0; i < 32; i++) lb[i] = i < 8 ? (uint8_t)(ml >> (8 * i)) : 0;
    chunk_ld(lw, lb);
    sha256_node(o, root, lw);
    LB_UNROLL for (int i = 0; i < 8; i++) root[i] = o[i];
  }
  chunk_st(roots + (size_t)32 * t, root);
}
#endif  // LB_KG
