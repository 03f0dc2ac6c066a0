// bih_packet_asm.h -- the packet walk of k_render_packet2 (bih_render.hip) as
// one hand-scheduled gfx950 loop (inline asm).
//
// Why asm: the walk is bound by wave-uniform (SALU) issue -- one scalar unit
// per CU serves every wave on it -- and hipcc's lowering of the uniform
// control flow (structurized branches, lane-mask booleans, stack arrays in
// scratch) spends about twice the scalar instructions of the sequence below.
// Semantics are exactly k_render_packet2's: same per-lane decisions, same
// f32 operations in the same order, same child order, same counters.
//
// Register map (physical registers, listed as clobbers so hipcc keeps its
// own values out of them; the stack lives only inside the statement):
//   s[36:39]  node record {d0, d1, z, w}            s[40:55]  triangle record
//   s[56:57]  act    s[58:59] gL   s[60:61] gR      s[62:63]  neg lanes (axis)
//   s[64:65]  tmp / triangle hit mask               s[66:67]  tmp / pickL mask
//   s[68:69]  left-leaf lanes  s[70:71] right-leaf lanes  s[72:73] tmp
//   s74 cur  s75 sp  s76 axis  s77 split  s78-s80 tmp  s81 b  s82 e
//   s83 saved m0  s84 mid  s85 near bit
//   s[88:95]  prefetched records of the current node's children (split, split+1)
//   v24 inv  v25 t0  v26 t1  v27 sL  v28 sR  v29-v32 {lo,hi} of left/right
//   v33-v38 temps (MT: v35-v37 p, v38 det then 1/det)  v39 stacked node ids
//   (lane k = slot k)  v40-v51 stacked lo (slot = gpr index)  v52-v63 stacked hi
// Slots >= BIH_ASM_SLOTS go to the wave's HBM spill area, [slot - BIH_ASM_SLOTS]
// x {lo[64], hi[64]} f32.  Lanes outside a stacked entry's mask hold the
// signalling-NaN pattern 0x7f800001 in lo (no f32 operation produces it).
#pragma once

#define BIH_ASM_SLOTS 12
#define BIH_S2(x) #x
#define BIH_S(x) BIH_S2(x)

// counters (STATS builds): v33 = this lane in MASK ? 1 : 0; counter += v33
#define BIH_CNT(MASK, CNT) "v_cndmask_b32_e64 v33, 0, 1, " MASK "\n\tv_add_u32_e32 %[" CNT "], v33, %[" CNT "]\n\t"

// Moeller-Trumbore of the record in s[40:55] for the lanes of MASK; the
// passing lanes end in s[64:65]; a uniform miss jumps to NEXT.
// Operand order of every f32 op follows prim_hits (bih_render.hip).
#define BIH_MT(MASK, NEXT)                                                            \
    "v_mul_f32_e32 v33, s45, %[dy]\n\t"      /* px = dy*e2z - e2y*dz */               \
    "v_mul_f32_e32 v34, s44, %[dz]\n\t"                                               \
    "v_sub_f32_e32 v35, v33, v34\n\t"                                                 \
    "v_mul_f32_e32 v33, s43, %[dz]\n\t"      /* py = dz*e2x - e2z*dx */               \
    "v_mul_f32_e32 v34, s45, %[dx]\n\t"                                               \
    "v_sub_f32_e32 v36, v33, v34\n\t"                                                 \
    "v_mul_f32_e32 v33, s44, %[dx]\n\t"      /* pz = dx*e2y - e2x*dy */               \
    "v_mul_f32_e32 v34, s43, %[dy]\n\t"                                               \
    "v_sub_f32_e32 v37, v33, v34\n\t"                                                 \
    "v_mul_f32_e32 v33, s40, v35\n\t"        /* det = (e1x*px + e1y*py) + e1z*pz */   \
    "v_mul_f32_e32 v34, s41, v36\n\t"                                                 \
    "v_add_f32_e32 v33, v33, v34\n\t"                                                 \
    "v_mul_f32_e32 v34, s42, v37\n\t"                                                 \
    "v_add_f32_e32 v38, v33, v34\n\t"                                                 \
    "v_cmp_nle_f32_e64 s[64:65], v38, %[eps]\n\t"   /* !(det <= eps): NaN passes */   \
    "s_and_b64 s[64:65], s[64:65], " MASK "\n\t"                                      \
    "s_cbranch_scc0 " NEXT "\n\t"                                                     \
    "v_div_scale_f32 v25, s[66:67], v38, v38, 1.0\n\t"   /* 1/det, IEEE (hipcc's */  \
    "v_rcp_f32_e32 v26, v25\n\t"                         /* own sequence)        */  \
    "v_div_scale_f32 v27, vcc, 1.0, v38, 1.0\n\t"                                     \
    "v_fma_f32 v28, -v25, v26, 1.0\n\t"                                               \
    "v_fmac_f32_e32 v26, v28, v26\n\t"                                                \
    "v_mul_f32_e32 v28, v27, v26\n\t"                                                 \
    "v_fma_f32 v24, -v25, v28, v27\n\t"                                               \
    "v_fmac_f32_e32 v28, v24, v26\n\t"                                                \
    "v_fma_f32 v25, -v25, v28, v27\n\t"                                               \
    "v_div_fmas_f32 v25, v25, v26, v28\n\t"                                           \
    "v_div_fixup_f32 v38, v25, v38, 1.0\n\t"                                          \
    "v_mul_f32_e32 v33, s46, v35\n\t"        /* u = ((sx*px + sy*py) + sz*pz)*inv */  \
    "v_mul_f32_e32 v34, s47, v36\n\t"                                                 \
    "v_add_f32_e32 v33, v33, v34\n\t"                                                 \
    "v_mul_f32_e32 v34, s48, v37\n\t"                                                 \
    "v_add_f32_e32 v33, v33, v34\n\t"                                                 \
    "v_mul_f32_e32 v35, v33, v38\n\t"                                                 \
    "v_cmp_nlt_f32_e64 s[66:67], v35, 0\n\t"        /* !(u < 0 || u > 1) */           \
    "v_cmp_ngt_f32_e64 s[72:73], v35, 1.0\n\t"                                        \
    "s_and_b64 s[64:65], s[64:65], s[66:67]\n\t"                                      \
    "s_and_b64 s[64:65], s[64:65], s[72:73]\n\t"                                      \
    "s_cbranch_scc0 " NEXT "\n\t"                                                     \
    "v_mul_f32_e32 v33, s49, %[dx]\n\t"      /* v = ((dx*qx + dy*qy) + dz*qz)*inv */  \
    "v_mul_f32_e32 v34, s50, %[dy]\n\t"                                               \
    "v_add_f32_e32 v33, v33, v34\n\t"                                                 \
    "v_mul_f32_e32 v34, s51, %[dz]\n\t"                                               \
    "v_add_f32_e32 v33, v33, v34\n\t"                                                 \
    "v_mul_f32_e32 v36, v33, v38\n\t"                                                 \
    "v_mul_f32_e32 v37, s52, v38\n\t"        /* t = tnum*inv */                       \
    "v_add_f32_e32 v33, v35, v36\n\t"        /* u + v */                              \
    "v_cmp_nlt_f32_e64 s[66:67], v36, 0\n\t"        /* !(v < 0 || u+v > 1) */         \
    "v_cmp_ngt_f32_e64 s[72:73], v33, 1.0\n\t"                                        \
    "s_and_b64 s[64:65], s[64:65], s[66:67]\n\t"                                      \
    "s_and_b64 s[64:65], s[64:65], s[72:73]\n\t"                                      \
    "v_cmp_lt_f32_e64 s[66:67], 0, v37\n\t"         /* t > 0 && t < FLT_MAX */        \
    "v_cmp_gt_f32_e64 s[72:73], %[fmax], v37\n\t"                                     \
    "s_and_b64 s[64:65], s[64:65], s[66:67]\n\t"                                      \
    "s_and_b64 s[64:65], s[64:65], s[72:73]\n\t"

// Triangles [s77, s82) for the lanes of MASK.
#define BIH_TRIS(TAG, MASK, ANY_MASK, CNT_TRI)                                        \
    ".LBIH_T" TAG "_%=:\n\t"                                                            \
    "s_cmp_ge_u32 s81, s82\n\t"                                                       \
    "s_cbranch_scc1 .LBIH_T" TAG "E_%=\n\t"                                             \
    ANY_MASK                                                                          \
    CNT_TRI                                                                           \
    "s_lshl_b32 s78, s81, 6\n\t"                                                      \
    "s_load_dwordx16 s[40:55], %[prims], s78\n\t"                                     \
    "s_add_u32 s81, s81, 1\n\t"                                                       \
    "s_waitcnt lgkmcnt(0)\n\t"                                                        \
    BIH_MT(MASK, ".LBIH_T" TAG "_%=")                                                   \
    "s_or_b64 %[hits], %[hits], s[64:65]\n\t"                                         \
    "s_branch .LBIH_T" TAG "_%=\n\t"                                                    \
    ".LBIH_T" TAG "E_%=:\n\t"

// Left leaf (triangles [mid - cL, mid), leaf index split) for s[68:69].
#define BIH_LEAF_L(TAG, ANY, CNT_LEAF, CNT_TRI)                                       \
    "s_cmp_eq_u64 s[68:69], 0\n\t"                                                    \
    "s_cbranch_scc1 .LBIH_LL" TAG "_%=\n\t"                                             \
    CNT_LEAF                                                                          \
    "s_bfe_u32 s79, s39, 0x2001b\n\t"        /* cntL, 0 = read dup_cnt */            \
    "s_cbranch_scc1 .LBIH_LC" TAG "_%=\n\t"                                             \
    "s_lshl_b32 s80, s77, 2\n\t"                                                      \
    "s_load_dword s79, %[dupc], s80\n\t"                                              \
    "s_waitcnt lgkmcnt(0)\n\t"                                                        \
    ".LBIH_LC" TAG "_%=:\n\t"                                                           \
    "s_sub_u32 s81, s84, s79\n\t"                                                     \
    "s_mov_b32 s82, s84\n\t"                                                          \
    BIH_TRIS("L" TAG, "s[68:69]", ANY("s[68:69]", ".LBIH_TL" TAG "E_%="), CNT_TRI)      \
    ".LBIH_LL" TAG "_%=:\n\t"

// Right leaf (triangles [mid, mid + cR), leaf index split + 1) for s[70:71].
#define BIH_LEAF_R(TAG, ANY, CNT_LEAF, CNT_TRI)                                       \
    "s_cmp_eq_u64 s[70:71], 0\n\t"                                                    \
    "s_cbranch_scc1 .LBIH_RR" TAG "_%=\n\t"                                             \
    CNT_LEAF                                                                          \
    "s_bfe_u32 s79, s39, 0x2001d\n\t"        /* cntR */                               \
    "s_cbranch_scc1 .LBIH_RC" TAG "_%=\n\t"                                             \
    "s_lshl_b32 s80, s77, 2\n\t"                                                      \
    "s_add_u32 s80, s80, 4\n\t"                                                       \
    "s_load_dword s79, %[dupc], s80\n\t"                                              \
    "s_waitcnt lgkmcnt(0)\n\t"                                                        \
    ".LBIH_RC" TAG "_%=:\n\t"                                                           \
    "s_mov_b32 s81, s84\n\t"                                                          \
    "s_add_u32 s82, s84, s79\n\t"                                                     \
    BIH_TRIS("R" TAG, "s[70:71]", ANY("s[70:71]", ".LBIH_TR" TAG "E_%="), CNT_TRI)      \
    ".LBIH_RR" TAG "_%=:\n\t"

// any-hit: drop lanes that already hit; leave when none is left
#define BIH_ANY_ON(MASK, EXIT) "s_andn2_b64 " MASK ", " MASK ", %[hits]\n\ts_cbranch_scc0 " EXIT "\n\t"
#define BIH_ANY_OFF(MASK, EXIT) ""
#define BIH_CLR_ON(MASK) "s_andn2_b64 " MASK ", " MASK ", %[hits]\n\t"
#define BIH_CLR_OFF(MASK) ""
// pop (any-hit): entry lanes that already hit drop out; all gone -> pop again
#define BIH_POP_ANY "s_andn2_b64 s[56:57], s[56:57], %[hits]\n\ts_cbranch_scc0 .LBIH_P_%=\n\t"
// STATS counters per walk event (act at a node, leaf lanes, triangle lanes)
#define BIH_CNT_NODE BIH_CNT("s[56:57]", "cn")
#define BIH_CNT_LEAF_L BIH_CNT("s[68:69]", "cl")
#define BIH_CNT_LEAF_R BIH_CNT("s[70:71]", "cl")
#define BIH_CNT_TRI_L BIH_CNT("s[68:69]", "ct")
#define BIH_CNT_TRI_R BIH_CNT("s[70:71]", "ct")

#define BIH_PACKET_WALK(ANY, CLR, ANY_TEXT, CNT_NODE, CNT_LEAF_L, CNT_LEAF_R, CNT_TRI_L, CNT_TRI_R) \
    "s_mov_b32 s83, m0\n\t"                                                           \
    "s_mov_b32 s74, 0\n\t"                                                            \
    "s_mov_b32 s75, 0\n\t"                                                            \
    "s_mov_b64 s[56:57], %[live]\n\t"                                                 \
    "s_mov_b64 %[hits], 0\n\t"                                                        \
    /* ---- node step: cur's record, per-lane child decisions ---- */                 \
    ".LBIH_N_%=:\n\t"                       /* cur's record from memory (root, pops) */ \
    CNT_NODE                                                                          \
    "s_lshl_b32 s78, s74, 4\n\t"                                                      \
    "s_load_dwordx4 s[36:39], %[nodes], s78\n\t"                                      \
    "s_waitcnt lgkmcnt(0)\n\t"                                                        \
    "s_branch .LBIH_NB_%=\n\t"                                                        \
    ".LBIH_NC_%=:\n\t"                      /* cur is a child of the last node: its */ \
    CNT_NODE                                 /* record was prefetched with its sibling */ \
    "s_waitcnt lgkmcnt(0)\n\t"                                                        \
    "s_cmp_eq_u32 s74, s77\n\t"                                                       \
    "s_cselect_b64 s[36:37], s[88:89], s[92:93]\n\t"                                  \
    "s_cselect_b64 s[38:39], s[90:91], s[94:95]\n\t"                                  \
    ".LBIH_NB_%=:\n\t"                                                                \
    "s_and_b32 s77, s38, 0x7ffffff\n\t"    /* split; prefetch nodes split, split+1 */ \
    "s_lshl_b32 s78, s77, 4\n\t"                                                      \
    "s_load_dwordx8 s[88:95], %[nodes], s78\n\t"                                      \
    "s_bitcmp1_b32 s38, 27\n\t"              /* inv = {ix, iy, iz}[axis] */           \
    "s_cselect_b64 s[64:65], -1, 0\n\t"                                               \
    "v_cndmask_b32_e64 v24, %[ix], %[iy], s[64:65]\n\t"                               \
    "s_bitcmp1_b32 s38, 28\n\t"                                                       \
    "s_cselect_b64 s[64:65], -1, 0\n\t"                                               \
    "v_cndmask_b32_e64 v24, v24, %[iz], s[64:65]\n\t"                                 \
    "s_bfe_u32 s76, s38, 0x2001b\n\t"                                                 \
    "v_bfe_u32 v33, %[sgn], s76, 1\n\t"      /* this lane runs -axis */               \
    "v_cmp_ne_u32_e64 s[62:63], 0, v33\n\t"                                           \
    "v_mul_f32_e32 v25, s36, v24\n\t"        /* t0 = (clip0 - O[axis]) * inv */       \
    "v_mul_f32_e32 v26, s37, v24\n\t"        /* t1 */                                 \
    "v_cndmask_b32_e64 v27, %[tmin], %[tmax], s[62:63]\n\t"                           \
    "v_cndmask_b32_e64 v28, %[tmax], %[tmin], s[62:63]\n\t"                           \
    "v_cmp_gt_f32_e64 s[58:59], v25, v27\n\t"                                         \
    "v_cmp_gt_f32_e64 s[60:61], v26, v28\n\t"                                         \
    "v_cndmask_b32_e64 v29, %[tmin], v25, s[62:63]\n\t"   /* left  [neg ? t0 : tMin, */ \
    "v_cndmask_b32_e64 v30, v25, %[tmax], s[62:63]\n\t"   /*        neg ? tMax : t0] */ \
    "v_cndmask_b32_e64 v31, v26, %[tmin], s[62:63]\n\t"   /* right [neg ? tMin : t1, */ \
    "v_cndmask_b32_e64 v32, %[tmax], v26, s[62:63]\n\t"   /*        neg ? t1 : tMax] */ \
    "s_xor_b64 s[58:59], s[58:59], s[62:63]\n\t"          /* gL = (t0 > sL) ^ neg */  \
    "s_and_b64 s[58:59], s[58:59], s[56:57]\n\t"                                      \
    "s_xnor_b64 s[60:61], s[60:61], s[62:63]\n\t"         /* gR = !((t1 > sR) ^ neg) */ \
    "s_and_b64 s[60:61], s[60:61], s[56:57]\n\t"                                      \
    "s_lshr_b32 s78, s38, 29\n\t"            /* leaf bits */                          \
    "s_cbranch_scc1 .LBIH_L_%=\n\t"                                                     \
    /* ---- descend: take near (majority order) or the only child, stack other ---- */ \
    ".LBIH_D_%=:\n\t"                                                                   \
    "s_or_b64 s[64:65], s[58:59], s[60:61]\n\t"                                       \
    "s_cbranch_scc0 .LBIH_P_%=\n\t"                                                     \
    "s_lshr_b32 s78, %[near], s76\n\t"                                                \
    "s_and_b32 s78, s78, 1\n\t"                                                       \
    "s_cmp_lg_u64 s[58:59], 0\n\t"                                                    \
    "s_cselect_b32 s79, 1, 0\n\t"                                                     \
    "s_cmp_eq_u64 s[60:61], 0\n\t"                                                    \
    "s_cselect_b32 s80, 1, 0\n\t"                                                     \
    "s_cmp_lg_u32 s78, 0\n\t"                                                         \
    "s_cselect_b32 s79, s79, s80\n\t"        /* pickL */                              \
    "s_cmp_lg_u32 s79, 0\n\t"                                                         \
    "s_cselect_b64 s[56:57], s[58:59], s[60:61]\n\t"                                  \
    "s_cselect_b64 s[64:65], s[60:61], s[58:59]\n\t"                                  \
    "s_cselect_b64 s[66:67], -1, 0\n\t"                                               \
    "s_add_u32 s80, s77, s79\n\t"            /* other = split + pickL */              \
    "s_xor_b32 s79, s79, 1\n\t"                                                       \
    "s_add_u32 s74, s77, s79\n\t"            /* taken = split + !pickL */             \
    "v_cndmask_b32_e64 %[tmin], v31, v29, s[66:67]\n\t"                               \
    "v_cndmask_b32_e64 %[tmax], v32, v30, s[66:67]\n\t"                               \
    "s_cmp_eq_u64 s[64:65], 0\n\t"                                                    \
    "s_cbranch_scc1 .LBIH_NC_%=\n\t"                                                    \
    "v_cndmask_b32_e64 v33, v29, v31, s[66:67]\n\t"                                   \
    "v_cndmask_b32_e64 v34, v30, v32, s[66:67]\n\t"                                   \
    "v_cndmask_b32_e64 v33, %[snan], v33, s[64:65]\n\t"                               \
    "s_cmp_ge_u32 s75, " BIH_S(BIH_ASM_SLOTS) "\n\t"                                  \
    "s_cbranch_scc1 .LBIH_SP_%=\n\t"                                                    \
    "s_set_gpr_idx_on s75, gpr_idx(DST)\n\t"                                          \
    "v_mov_b32_e32 v40, v33\n\t"                                                      \
    "v_mov_b32_e32 v52, v34\n\t"                                                      \
    "s_set_gpr_idx_off\n\t"                                                           \
    ".LBIH_PN_%=:\n\t"                                                                  \
    "s_mov_b32 m0, s75\n\t"                                                          \
    "s_nop 0\n\t"                                                                     \
    "v_writelane_b32 v39, s80, m0\n\t"                                               \
    "s_add_u32 s75, s75, 1\n\t"                                                       \
    "s_branch .LBIH_NC_%=\n\t"                                                          \
    ".LBIH_SP_%=:\n\t"                         /* deep slot: wave spill area */         \
    "s_sub_u32 s78, s75, " BIH_S(BIH_ASM_SLOTS) "\n\t"                                \
    "s_lshl_b32 s78, s78, 9\n\t"                                                      \
    "v_add_u32_e32 v35, s78, %[lane4]\n\t"                                            \
    "global_store_dword v35, v33, %[spill]\n\t"                                       \
    "global_store_dword v35, v34, %[spill] offset:256\n\t"                            \
    "s_waitcnt vmcnt(0)\n\t"                                                          \
    "s_branch .LBIH_PN_%=\n\t"                                                          \
    /* ---- pop until an entry has a searching lane ---- */                           \
    ".LBIH_P_%=:\n\t"                                                                   \
    "s_cmp_eq_u32 s75, 0\n\t"                                                         \
    "s_cbranch_scc1 .LBIH_X_%=\n\t"                                                     \
    "s_sub_u32 s75, s75, 1\n\t"                                                       \
    "s_cmp_ge_u32 s75, " BIH_S(BIH_ASM_SLOTS) "\n\t"                                  \
    "s_cbranch_scc1 .LBIH_SQ_%=\n\t"                                                    \
    "s_set_gpr_idx_on s75, gpr_idx(SRC0)\n\t"                                         \
    "v_mov_b32_e32 %[tmin], v40\n\t"                                                  \
    "v_mov_b32_e32 %[tmax], v52\n\t"                                                  \
    "s_set_gpr_idx_off\n\t"                                                           \
    ".LBIH_PQ_%=:\n\t"                                                                  \
    "s_nop 0\n\t"                                                                     \
    "v_readlane_b32 s74, v39, s75\n\t"                                                \
    "v_cmp_ne_u32_e64 s[56:57], %[snan], %[tmin]\n\t"                                 \
    ANY_TEXT                                                                          \
    "s_nop 1\n\t"                                                                     \
    "s_branch .LBIH_N_%=\n\t"                                                           \
    ".LBIH_SQ_%=:\n\t"                                                                  \
    "s_sub_u32 s78, s75, " BIH_S(BIH_ASM_SLOTS) "\n\t"                                \
    "s_lshl_b32 s78, s78, 9\n\t"                                                      \
    "v_add_u32_e32 v35, s78, %[lane4]\n\t"                                            \
    "global_load_dword %[tmin], v35, %[spill]\n\t"                                    \
    "global_load_dword %[tmax], v35, %[spill] offset:256\n\t"                         \
    "s_waitcnt vmcnt(0)\n\t"                                                          \
    "s_branch .LBIH_PQ_%=\n\t"                                                          \
    /* ---- leaves of this node: test them (near first), then descend ---- */         \
    ".LBIH_L_%=:\n\t"                                                                   \
    "s_bitcmp1_b32 s38, 29\n\t"                                                       \
    "s_cselect_b64 s[68:69], s[58:59], 0\n\t"                                         \
    "s_cselect_b64 s[58:59], 0, s[58:59]\n\t"                                         \
    "s_bitcmp1_b32 s38, 30\n\t"                                                       \
    "s_cselect_b64 s[70:71], s[60:61], 0\n\t"                                         \
    "s_cselect_b64 s[60:61], 0, s[60:61]\n\t"                                         \
    "s_and_b32 s84, s39, 0x7ffffff\n\t"                                               \
    "s_lshr_b32 s85, %[near], s76\n\t"                                                \
    "s_bitcmp1_b32 s85, 0\n\t"                                                        \
    "s_cbranch_scc0 .LBIH_LR_%=\n\t"                                                    \
    BIH_LEAF_L("a", ANY, CNT_LEAF_L, CNT_TRI_L)                                       \
    BIH_LEAF_R("a", ANY, CNT_LEAF_R, CNT_TRI_R)                                       \
    "s_branch .LBIH_LE_%=\n\t"                                                          \
    ".LBIH_LR_%=:\n\t"                                                                  \
    BIH_LEAF_R("b", ANY, CNT_LEAF_R, CNT_TRI_R)                                       \
    BIH_LEAF_L("b", ANY, CNT_LEAF_L, CNT_TRI_L)                                       \
    ".LBIH_LE_%=:\n\t"                                                                  \
    CLR("s[58:59]")                                                                   \
    CLR("s[60:61]")                                                                   \
    "s_branch .LBIH_D_%=\n\t"                                                           \
    ".LBIH_X_%=:\n\t"                                                                   \
    "s_mov_b32 m0, s83"

#define BIH_PACKET_CLOBBERS                                                           \
    "s36", "s37", "s38", "s39", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", \
    "s48", "s49", "s50", "s51", "s52", "s53", "s54", "s55", "s56", "s57", "s58", "s59", \
    "s60", "s61", "s62", "s63", "s64", "s65", "s66", "s67", "s68", "s69", "s70", "s71", \
    "s72", "s73", "s74", "s75", "s76", "s77", "s78", "s79", "s80", "s81", "s82", "s83", \
    "s84", "s85", "s88", "s89", "s90", "s91", "s92", "s93", "s94", "s95",             \
    "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", \
    "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", \
    "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", \
    "v60", "v61", "v62", "v63", "vcc", "scc", "memory"
