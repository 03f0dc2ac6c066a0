// bih_packet_asm.h -- the packet walk of k_render_packet2 (bih_render.hip) as
// one hand-scheduled gfx950 loop (inline asm).
//
// Why asm: the walk is bound by wave-uniform issue -- one scalar ALU per CU
// serves every wave on it -- and hipcc's lowering of the uniform control flow
// (structurized branches, lane-mask booleans, stack arrays in scratch) spends
// several times the scalar instructions of the loop below.  The loop keeps
// the scalar unit for what only it can do (addresses, loads, 64-lane masks,
// branches) and moves selects and compares to the VALU, which has 4x the
// issue rate and is otherwise idle here.
//
// Semantics are exactly k_render_packet2's: the same per-lane decisions, the
// same f32 operations in the same order, the same child order, the same
// counters (tests/test_gpu_parity.py compares both kernels with the oracle).
//
// Node records come from the child-pair prefetch: at every node with two
// internal children the records of its children {split, split+1} are
// requested with one s_load_dwordx8 into the other of two record buffers
// (A = s[76:83], B = s[36:43]) before the node's decisions are computed;
// descending to the left child continues at NB<buf>0, to the right at
// NB<buf>1.  The root loads its record into A0 = s[76:79]; a pop reads it
// there from the VGPR stack (BIH_STACK_REC) or loads it like the root.
//
// Register map (physical registers, listed as clobbers so hipcc keeps its own
// values out of them; the stack lives only inside the statement).  Kept at or
// below s83 so the kernel stays within 96 SGPRs (7 waves per SIMD; the SGPR
// file holds 800 per SIMD, allocated in 16s plus 16 -- MI355X_MICROARCH.md):
//   s[36:51] triangle record; its first 8 also record buffer B (a node with a
//            leaf child never has a B prefetch in flight)
//   s[52:53] gL   s[54:55] gR   s[56:57] lanes running -axis
//   s[58:59] left-leaf lanes    s[60:61] right-leaf lanes    EXEC = active lanes
//   s62 cur (pop)  s63 sp  s64 pair offset  s65-s67 tmp  s68 b  s69 e
//   s70 saved m0  s71 w (mid | leaf bits | counts)  s72 leaf bits  s73 mid
//   s[76:83] record buffer A        M0[7:0] the node's axis until a push
//   v62-v64 {ix, iy, iz} (inv = v[62 + axis], gpr-indexed)
//   v24 inv  v25 t0  v26 t1  v27 sL  v28 sR  v29-v32 {lo,hi} of a stacked child
//   (MT: v24, v27-v30 division temps; t0/t1 survive the leaf tests)
//   v33-v38 temps (MT: v35-v37 p, v38 det then 1/det)  v39 stacked node ids
//   (lane k = slot k; BIH_STACK_REC: v39/v65/v66/v67 lane k = the 4 dwords of
//   slot k's record)  v40-v50 stacked lo (slot = gpr index)  v51-v61 stacked hi
//   (11 slots)
// Slots >= BIH_ASM_SLOTS go to the wave's HBM spill area, [slot - BIH_ASM_SLOTS]
// x {lo[64], hi[64]} f32.  Lanes outside a stacked entry's mask hold the
// signalling-NaN pattern 0x7f800001 in lo (no f32 operation produces it).
#pragma once

#define BIH_ASM_SLOTS 11
#define BIH_S2(x) #x
#define BIH_S(x) BIH_S2(x)

// counters (STATS builds): counter += 1 on the lanes of EXEC (the node's
// active lanes at a node step, the lanes testing the triangle in the leaf
// loop); a leaf counts the lanes of its mask
#define BIH_CNT_EXEC(CNT) "v_add_u32_e32 %[" CNT "], 1, %[" CNT "]\n\t"
#define BIH_CNT_MASK(MASK, CNT) "s_mov_b64 exec, " MASK "\n\t" BIH_CNT_EXEC(CNT)
#define BIH_CNT_NODE BIH_CNT_EXEC("cn")
#define BIH_CNT_LEAF_L BIH_CNT_MASK("s[58:59]", "cl")
#define BIH_CNT_LEAF_R BIH_CNT_MASK("s[60:61]", "cl")
#define BIH_CNT_TRI_L BIH_CNT_EXEC("ct")
#define BIH_CNT_TRI_R BIH_CNT_EXEC("ct")

// EXEC = the lanes testing the next triangle of a leaf: its mask, and with
// any-hit without the lanes that already hit (leave when none is left)
#define BIH_ANY_ON(MASK, EXIT) "s_andn2_b64 exec, " MASK ", %[hits]\n\ts_cbranch_scc0 " EXIT "\n\t"
#define BIH_ANY_OFF(MASK, EXIT) "s_mov_b64 exec, " MASK "\n\t"
#define BIH_CLR_ON(MASK) "s_andn2_b64 " MASK ", " MASK ", %[hits]\n\t"
#define BIH_CLR_OFF(MASK) ""
#define BIH_POP_ANY "s_andn2_b64 exec, exec, %[hits]\n\ts_cbranch_scc0 .LBIH_PL_%=\n\t"

// Moeller-Trumbore of the record in s[36:51] for the lanes of EXEC; each
// test narrows EXEC (v_cmpx), so the passing lanes end in EXEC; a uniform
// miss jumps to NEXT.
// Before the division, lanes whose u is certain to fail are dropped on the
// numerator un = dot(s, p) alone: with det in (eps, inf) finite, 1/det and
// un*(1/det) are each correctly rounded (relative error <= 2^-24), so
//   un < -det*2^-20     gives u <= (un/det)(1 - 2^-23) < -2^-21: u < 0;
//   un > det*(1+2^-20)  (the bound itself rounded by <= 2^-24) gives
//                       u >= (1+2^-20)(1-2^-24)^3 > 1: u > 1;
// det*2^-20 is exact (det > eps, no underflow); det = inf or NaN and un =
// NaN compare false and keep the lane.  The lanes kept run the exact test.
// Operand order of every f32 op follows prim_hits (bih_render.hip):
// record = {e1 s36-38, e2 s39-41, s = O - v0 s42-44, q s45-47, tnum s48}.
#define BIH_MT(NEXT)                                                                  \
    "v_mul_f32_e32 v33, s41, %[dy]\n\t"      /* px = dy*e2z - e2y*dz */               \
    "v_mul_f32_e32 v34, s40, %[dz]\n\t"                                               \
    "v_sub_f32_e32 v35, v33, v34\n\t"                                                 \
    "v_mul_f32_e32 v33, s39, %[dz]\n\t"      /* py = dz*e2x - e2z*dx */               \
    "v_mul_f32_e32 v34, s41, %[dx]\n\t"                                               \
    "v_sub_f32_e32 v36, v33, v34\n\t"                                                 \
    "v_mul_f32_e32 v33, s40, %[dx]\n\t"      /* pz = dx*e2y - e2x*dy */               \
    "v_mul_f32_e32 v34, s39, %[dy]\n\t"                                               \
    "v_sub_f32_e32 v37, v33, v34\n\t"                                                 \
    "v_mul_f32_e32 v33, s36, v35\n\t"        /* det = (e1x*px + e1y*py) + e1z*pz */   \
    "v_mul_f32_e32 v34, s37, v36\n\t"                                                 \
    "v_add_f32_e32 v33, v33, v34\n\t"                                                 \
    "v_mul_f32_e32 v34, s38, v37\n\t"                                                 \
    "v_add_f32_e32 v38, v33, v34\n\t"                                                 \
    "v_cmpx_nge_f32_e32 vcc, %[eps], v38\n\t"   /* !(det <= eps): NaN passes */        \
    "s_cbranch_execz " NEXT "\n\t"                                                    \
    "v_mul_f32_e32 v33, s42, v35\n\t"        /* un = (sx*px + sy*py) + sz*pz */        \
    "v_mul_f32_e32 v34, s43, v36\n\t"                                                 \
    "v_add_f32_e32 v33, v33, v34\n\t"                                                 \
    "v_mul_f32_e32 v34, s44, v37\n\t"                                                 \
    "v_add_f32_e32 v33, v33, v34\n\t"                                                 \
    /* division-free pre-test (see BIH_MT's comment): drop lanes with */              \
    /* un < -det*2^-20 (u < 0) or un > det*(1+2^-20) (u > 1) */                      \
    "v_mul_f32_e32 v34, 0x35800000, v38\n\t"                                          \
    "v_cmpx_nlt_f32_e64 vcc, v33, -v34\n\t"                                      \
    "v_mul_f32_e32 v34, 0x3f800008, v38\n\t"                                          \
    "v_cmpx_ngt_f32_e32 vcc, v33, v34\n\t"                                            \
    "s_cbranch_execz " NEXT "\n\t"                                                    \
    "v_div_scale_f32 v27, vcc, v38, v38, 1.0\n\t"   /* 1/det, IEEE (hipcc's */  \
    "v_rcp_f32_e32 v28, v27\n\t"                         /* own sequence; keeps  */  \
    "v_div_scale_f32 v29, vcc, 1.0, v38, 1.0\n\t"         /* t0/t1 in v25/v26)    */  \
    "v_fma_f32 v30, -v27, v28, 1.0\n\t"                                               \
    "v_fmac_f32_e32 v28, v30, v28\n\t"                                                \
    "v_mul_f32_e32 v30, v29, v28\n\t"                                                 \
    "v_fma_f32 v24, -v27, v30, v29\n\t"                                               \
    "v_fmac_f32_e32 v30, v24, v28\n\t"                                                \
    "v_fma_f32 v27, -v27, v30, v29\n\t"                                               \
    "v_div_fmas_f32 v27, v27, v28, v30\n\t"                                           \
    "v_div_fixup_f32 v38, v27, v38, 1.0\n\t"                                          \
    "v_mul_f32_e32 v35, v33, v38\n\t"        /* u = un * inv */                       \
    "v_cmpx_ngt_f32_e32 vcc, 0, v35\n\t"           /* !(u < 0 || u > 1) */            \
    "v_cmpx_nlt_f32_e32 vcc, 1.0, v35\n\t"                                            \
    "s_cbranch_execz " NEXT "\n\t"                                                    \
    "v_mul_f32_e32 v33, s45, %[dx]\n\t"      /* v = ((dx*qx + dy*qy) + dz*qz)*inv */  \
    "v_mul_f32_e32 v34, s46, %[dy]\n\t"                                               \
    "v_add_f32_e32 v33, v33, v34\n\t"                                                 \
    "v_mul_f32_e32 v34, s47, %[dz]\n\t"                                               \
    "v_add_f32_e32 v33, v33, v34\n\t"                                                 \
    "v_mul_f32_e32 v36, v33, v38\n\t"                                                 \
    "v_mul_f32_e32 v37, s48, v38\n\t"        /* t = tnum*inv */                       \
    "v_add_f32_e32 v33, v35, v36\n\t"        /* u + v */                              \
    "v_cmpx_ngt_f32_e32 vcc, 0, v36\n\t"           /* !(v < 0 || u+v > 1) */          \
    "v_cmpx_nlt_f32_e32 vcc, 1.0, v33\n\t"                                            \
    "v_cmpx_lt_f32_e32 vcc, 0, v37\n\t"            /* t > 0 && t < FLT_MAX */         \
    "v_cmpx_gt_f32_e32 vcc, %[fmax], v37\n\t"

// Triangles [s77, s78), at least one, for the lanes of the leaf's mask
// (ANY_MASK sets EXEC per triangle).
#define BIH_TRIS(TAG, ANY_MASK, CNT_TRI)                                              \
    ".LBIH_T" TAG "_%=:\n\t"                                                          \
    ANY_MASK                                                                          \
    CNT_TRI                                                                           \
    "s_lshl_b32 s65, s68, 6\n\t"                                                      \
    "s_load_dwordx16 s[36:51], %[prims], s65\n\t"                                     \
    "s_add_u32 s68, s68, 1\n\t"                                                       \
    "s_waitcnt lgkmcnt(0)\n\t"                                                        \
    BIH_MT(".LBIH_TN" TAG "_%=")                                                      \
    "s_or_b64 %[hits], %[hits], exec\n\t"                                             \
    ".LBIH_TN" TAG "_%=:\n\t"                                                         \
    "s_cmp_lt_u32 s68, s69\n\t"                                                       \
    "s_cbranch_scc1 .LBIH_T" TAG "_%=\n\t"                                            \
    ".LBIH_T" TAG "E_%=:\n\t"

// The one triangle at byte offset s74 (a leaf of count code 1, most leaves).
#define BIH_TRI1(ANY_MASK, CNT_TRI, EXIT)                                             \
    ANY_MASK                                                                          \
    CNT_TRI                                                                           \
    "s_load_dwordx16 s[36:51], %[prims], s65\n\t"                                     \
    "s_waitcnt lgkmcnt(0)\n\t"                                                        \
    BIH_MT(EXIT)                                                                      \
    "s_or_b64 %[hits], %[hits], exec\n\t"                                             \
    "s_branch " EXIT "\n\t"

// Left leaf (triangles [mid - cL, mid), leaf index split) for s[64:65].
#define BIH_LEAF_L(TAG, ANY, CNT_LEAF, CNT_TRI)                                       \
    "s_cmp_eq_u64 s[58:59], 0\n\t"                                                    \
    "s_cbranch_scc1 .LBIH_LL" TAG "_%=\n\t"                                           \
    CNT_LEAF                                                                          \
    "s_bfe_u32 s66, s71, 0x2001b\n\t"        /* cntL, 0 = read dup_cnt */            \
    "s_cbranch_scc0 .LBIH_LD" TAG "_%=\n\t"                                           \
    "s_cmp_eq_u32 s66, 1\n\t"                                                         \
    "s_cbranch_scc0 .LBIH_LC" TAG "_%=\n\t"                                           \
    "s_lshl_b32 s65, s73, 6\n\t"            /* triangle mid - 1 */                   \
    "s_sub_u32 s65, s65, 64\n\t"                                                      \
    BIH_TRI1(ANY("s[58:59]", ".LBIH_LL" TAG "_%="), CNT_TRI, ".LBIH_LL" TAG "_%=")     \
    ".LBIH_LD" TAG "_%=:\n\t"                                                         \
    "s_lshr_b32 s67, s64, 2\n\t"            /* split * 4 */                          \
    "s_load_dword s66, %[dupc], s67\n\t"                                              \
    "s_waitcnt lgkmcnt(0)\n\t"                                                        \
    ".LBIH_LC" TAG "_%=:\n\t"                                                         \
    "s_sub_u32 s68, s73, s66\n\t"                                                     \
    "s_mov_b32 s69, s73\n\t"                                                          \
    BIH_TRIS("L" TAG, ANY("s[58:59]", ".LBIH_TL" TAG "E_%="), CNT_TRI)                \
    ".LBIH_LL" TAG "_%=:\n\t"

// Right leaf (triangles [mid, mid + cR), leaf index split + 1) for s[66:67].
#define BIH_LEAF_R(TAG, ANY, CNT_LEAF, CNT_TRI)                                       \
    "s_cmp_eq_u64 s[60:61], 0\n\t"                                                    \
    "s_cbranch_scc1 .LBIH_RR" TAG "_%=\n\t"                                           \
    CNT_LEAF                                                                          \
    "s_bfe_u32 s66, s71, 0x2001d\n\t"        /* cntR */                               \
    "s_cbranch_scc0 .LBIH_RD" TAG "_%=\n\t"                                           \
    "s_cmp_eq_u32 s66, 1\n\t"                                                         \
    "s_cbranch_scc0 .LBIH_RC" TAG "_%=\n\t"                                           \
    "s_lshl_b32 s65, s73, 6\n\t"            /* triangle mid */                       \
    BIH_TRI1(ANY("s[60:61]", ".LBIH_RR" TAG "_%="), CNT_TRI, ".LBIH_RR" TAG "_%=")     \
    ".LBIH_RD" TAG "_%=:\n\t"                                                         \
    "s_lshr_b32 s67, s64, 2\n\t"                                                      \
    "s_add_u32 s67, s67, 4\n\t"                                                       \
    "s_load_dword s66, %[dupc], s67\n\t"                                              \
    "s_waitcnt lgkmcnt(0)\n\t"                                                        \
    ".LBIH_RC" TAG "_%=:\n\t"                                                         \
    "s_mov_b32 s68, s73\n\t"                                                          \
    "s_add_u32 s69, s73, s66\n\t"                                                     \
    BIH_TRIS("R" TAG, ANY("s[60:61]", ".LBIH_TR" TAG "E_%="), CNT_TRI)                \
    ".LBIH_RR" TAG "_%=:\n\t"

// Consume the node record (d0 d1 z w in 4 SGPRs, z = split << 8 | axis, w =
// mid | leafL << 26 | cntL << 27 | cntR << 29 | leafR << 31): the lane's inv
// and -axis mask (VALU), t0/t1.  s_set_gpr_idx_on takes the index from z's
// low byte (= axis) and leaves it in M0[7:0], where the near-order tests of
// this node read it (bit M0[4:0] of %[near]) until a push rewrites M0.
#define BIH_NODE_REC(D0, D1, Z)                                                       \
    "s_set_gpr_idx_on " Z ", gpr_idx(SRC0)\n\t"                                       \
    "v_mov_b32_e32 v24, v62\n\t"            /* inv = {ix,iy,iz}[axis] (v62-v64) */    \
    "s_set_gpr_idx_off\n\t"                                                          \
    "v_cmp_gt_f32_e64 s[56:57], 0, v24\n\t" /* this lane runs -axis: sign = inv < 0 */ \
    "v_mul_f32_e32 v25, " D0 ", v24\n\t"     /* t0 = (clip0 - O[axis]) * inv */       \
    "v_mul_f32_e32 v26, " D1 ", v24\n\t"     /* t1 */

// Per-lane child decisions (EXEC = the node's lanes; compares give 0 off
// EXEC).  s[54:55] / s[56:57] leave here as the raw compares; gL = s[54:55] ^
// neg is formed before D (SCC = gL != 0), gR = s[56:57] ^ neg where it is
// first tested (its SCC then replaces a compare with 0).
#define BIH_NODE_DEC                                                                  \
    "v_cndmask_b32_e64 v27, %[tmin], %[tmax], s[56:57]\n\t"   /* sL = neg ? tMax : tMin */ \
    "v_cndmask_b32_e64 v28, %[tmax], %[tmin], s[56:57]\n\t"   /* sR = neg ? tMin : tMax */ \
    "v_cmp_gt_f32_e64 s[52:53], v25, v27\n\t"                                         \
    "v_cmp_ngt_f32_e64 s[54:55], v26, v28\n\t"

// Node step of the record {D0 D1 Z W} held in one half of a record buffer.
// Two internal children: their record pair is requested into the OTHER
// buffer (YREGS) before the decisions are computed, so the load overlaps
// them, and the walk continues at D<DY> (DTAIL: a branch, or nothing where
// D<DY> follows).  A leaf child: LV<TAG> (out of line, BIH_NODE_LV).
#define BIH_NODE_STEP(TAG, CNT_NODE, D0, D1, Z, W, YREGS, DTAIL)                       \
    ".LBIH_NB" TAG "_%=:\n\t"                                                         \
    CNT_NODE                                                                          \
    "s_lshr_b32 s64, " Z ", 4\n\t"           /* byte offset of the children's pair */ \
    "s_and_b32 s72, " W ", 0x84000000\n\t"  /* leaf bits: 1<<26 left, 1<<31 right */  \
    "s_cbranch_scc1 .LBIH_LV" TAG "_%=\n\t"                                           \
    "s_load_dwordx8 " YREGS ", %[nodes], s64\n\t"                                     \
    BIH_NODE_REC(D0, D1, Z)                                                           \
    BIH_NODE_DEC                                                                      \
    "s_xor_b64 s[52:53], s[52:53], s[56:57]\n\t"  /* gL = (t0 > sL) ^ neg; SCC = gL != 0 */ \
    DTAIL

// The same node step when a child is a leaf: decisions, w to s80, then the
// shared leaf section L.
#define BIH_NODE_LV(TAG, D0, D1, Z, W)                                                \
    ".LBIH_LV" TAG "_%=:\n\t"                                                         \
    BIH_NODE_REC(D0, D1, Z)                                                           \
    BIH_NODE_DEC                                                                      \
    "s_xor_b64 s[52:53], s[52:53], s[56:57]\n\t"          /* gL */                    \
    "s_xor_b64 s[54:55], s[54:55], s[56:57]\n\t"          /* gR */                    \
    "s_mov_b32 s71, " W "\n\t"               /* w: mid | leaf bits | counts */         \
    "s_branch .LBIH_L_%=\n\t"

// Descend with the children's records in buffer Y (Y0 = left, Y1 = right):
// the near child (majority order) if visited, the other stacked.
#define BIH_DESCEND(Y, RECL, RECR)                                                                \
    ".LBIH_D" Y "_%=:\n\t"                   /* SCC = (gL != 0) */                     \
    "s_cbranch_scc0 .LBIH_DN" Y "_%=\n\t"                                             \
    "s_xor_b64 s[54:55], s[54:55], s[56:57]\n\t"  /* gR = !(t1 > sR) ^ neg; SCC = gR != 0 */ \
    "s_cbranch_scc0 .LBIH_TL" Y "_%=\n\t"    /* only the left child */                \
    "s_bitcmp1_b32 %[near], m0\n\t"         /* both: near first, stack the other */  \
    "s_cbranch_scc0 .LBIH_BR" Y "_%=\n\t"                                             \
    "v_cndmask_b32_e64 v31, v26, %[tmin], s[56:57]\n\t"   /* right [neg ? tMin : t1, */ \
    "v_cndmask_b32_e64 v32, %[tmax], v26, s[56:57]\n\t"   /*        neg ? t1 : tMax] */ \
    BIH_PUSH("r" Y, "s[54:55]", "v31", "v32", "s_add_u32 s65, s64, 16\n\t", "s65", RECR)  \
    ".LBIH_TL" Y "_%=:\n\t"                  /* take left: record in Y0 */             \
    "s_mov_b64 exec, s[52:53]\n\t"                                                    \
    "v_cndmask_b32_e64 %[tmin], %[tmin], v25, s[56:57]\n\t" /* [neg ? t0 : tMin,    */ \
    "v_cndmask_b32_e64 %[tmax], v25, %[tmax], s[56:57]\n\t" /*  neg ? tMax : t0]    */ \
    "s_waitcnt lgkmcnt(0)\n\t"                                                        \
    "s_branch .LBIH_NB" Y "0_%=\n\t"                                                  \
    ".LBIH_BR" Y "_%=:\n\t"                                                           \
    "v_cndmask_b32_e64 v29, %[tmin], v25, s[56:57]\n\t"   /* left  [neg ? t0 : tMin, */ \
    "v_cndmask_b32_e64 v30, v25, %[tmax], s[56:57]\n\t"   /*        neg ? tMax : t0] */ \
    BIH_PUSH("l" Y, "s[52:53]", "v29", "v30", "", "s64", RECL)                              \
    ".LBIH_TR" Y "_%=:\n\t"                  /* take right: record in Y1 */            \
    "s_mov_b64 exec, s[54:55]\n\t"                                                    \
    "v_cndmask_b32_e64 %[tmin], v26, %[tmin], s[56:57]\n\t" /* [neg ? tMin : t1,    */ \
    "v_cndmask_b32_e64 %[tmax], %[tmax], v26, s[56:57]\n\t" /*  neg ? t1 : tMax]    */ \
    "s_waitcnt lgkmcnt(0)\n\t"                                                        \
    "s_branch .LBIH_NB" Y "1_%=\n\t"                                                  \
    ".LBIH_DN" Y "_%=:\n\t"                  /* no left: right or pop */              \
    "s_xor_b64 s[54:55], s[54:55], s[56:57]\n\t"  /* gR; SCC = gR != 0 */             \
    "s_cbranch_scc1 .LBIH_TR" Y "_%=\n\t"                                             \
    "s_branch .LBIH_P_%=\n\t"

// Stack entry {lane lo/hi (sentinel outside MASK), node = NODE, the byte
// offset of its record (NODE_SET forms it in s74 where it is not s73)};
// written on every lane (EXEC = all; the caller sets EXEC afterwards).
// s_set_gpr_idx_on leaves the slot index in M0[7:0], the lane v_writelane
// selects.  Deep slots go to the wave's spill area in the out-of-line block
// BIH_PUSH_SPILL(TAG) emits (which sets M0 itself).
#define BIH_PUSH(TAG, MASK, LO, HI, NODE_SET, NODE, R)                                \
    "s_mov_b64 exec, -1\n\t"                                                          \
    "v_cndmask_b32_e64 v33, %[snan], " LO ", " MASK "\n\t"                            \
    "s_cmp_ge_u32 s63, " BIH_S(BIH_ASM_SLOTS) "\n\t"                                  \
    "s_cbranch_scc1 .LBIH_SP" TAG "_%=\n\t"                                           \
    "s_set_gpr_idx_on s63, gpr_idx(DST)\n\t"                                          \
    "v_mov_b32_e32 v40, v33\n\t"                                                      \
    "v_mov_b32_e32 v51, " HI "\n\t"                                                   \
    "s_set_gpr_idx_off\n\t"                                                           \
    ".LBIH_PN" TAG "_%=:\n\t"                                                         \
    BIH_PUSH_NODE(NODE_SET, NODE, R)                                                  \
    "s_add_u32 s63, s63, 1\n\t"

// The stacked node itself.  BIH_STACK_REC: its whole 16-byte record (already
// in the pair buffer, R = its 4 SGPRs) goes to lane <slot> of v39/v65/v66/v67,
// so a pop reads it back with v_readlane and starts the node step without a
// load.  Else: its byte offset to lane <slot> of v39, and the pop loads it.
#ifndef BIH_STACK_REC
#define BIH_STACK_REC 0
#endif
#if BIH_STACK_REC
#define BIH_PUSH_NODE(NODE_SET, NODE, R) R
#define BIH_REC(R0, R1, R2, R3)                                                       \
    "s_waitcnt lgkmcnt(0)\n\t"               /* the pair prefetch has landed */       \
    "v_writelane_b32 v39, " R0 ", m0\n\t"                                             \
    "v_writelane_b32 v65, " R1 ", m0\n\t"                                             \
    "v_writelane_b32 v66, " R2 ", m0\n\t"                                             \
    "v_writelane_b32 v67, " R3 ", m0\n\t"
#define BIH_REC_CLOBBERS "v65", "v66", "v67",
// Pop: EXEC = the entry's lanes, then its record straight into buffer A
// (v_readlane ignores EXEC) and the node step A0.
#define BIH_POP_NODE(ANY_TEXT)                                                        \
    "s_nop 0\n\t"                                                                     \
    "v_cmpx_ne_u32_e32 vcc, %[snan], %[tmin]\n\t"  /* EXEC = the entry's lanes */      \
    ANY_TEXT                                                                          \
    "v_readlane_b32 s76, v39, s63\n\t"                                                \
    "v_readlane_b32 s77, v65, s63\n\t"                                                \
    "v_readlane_b32 s78, v66, s63\n\t"                                                \
    "v_readlane_b32 s79, v67, s63\n\t"                                                \
    "s_nop 1\n\t"                                                                     \
    "s_branch .LBIH_NBA0_%=\n\t"
#else
#define BIH_PUSH_NODE(NODE_SET, NODE, R) NODE_SET "v_writelane_b32 v39, " NODE ", m0\n\t"
#define BIH_REC(R0, R1, R2, R3) ""
#define BIH_REC_CLOBBERS
// Pop: EXEC = the entry's lanes, its record's offset for the load at N.
#define BIH_POP_NODE(ANY_TEXT)                                                        \
    "s_nop 0\n\t"                                                                     \
    "v_readlane_b32 s62, v39, s63\n\t"                                                \
    "v_cmpx_ne_u32_e32 vcc, %[snan], %[tmin]\n\t"  /* EXEC = the entry's lanes */      \
    ANY_TEXT                                                                          \
    "s_nop 1\n\t"                                                                     \
    "s_branch .LBIH_N_%=\n\t"
#endif

#define BIH_PUSH_SPILL(TAG, HI)                                                       \
    ".LBIH_SP" TAG "_%=:\n\t"                /* deep slot: wave spill area */         \
    "s_mov_b32 m0, s63\n\t"                  /* the lane v_writelane selects */     \
    "s_sub_u32 s65, s63, " BIH_S(BIH_ASM_SLOTS) "\n\t"                                \
    "s_lshl_b32 s65, s65, 9\n\t"                                                      \
    "v_add_u32_e32 v35, s65, %[lane4]\n\t"                                            \
    "global_store_dword v35, v33, %[spill]\n\t"                                       \
    "global_store_dword v35, " HI ", %[spill] offset:256\n\t"                         \
    "s_waitcnt vmcnt(0)\n\t"                                                          \
    "s_branch .LBIH_PN" TAG "_%=\n\t"

#define BIH_PACKET_WALK(ANY, CLR, ANY_TEXT, CNT_NODE, CNT_LEAF_L, CNT_LEAF_R, CNT_TRI_L, CNT_TRI_R) \
    "s_mov_b32 s70, m0\n\t"                                                           \
    "v_mov_b32_e32 v62, %[ix]\n\t"                                                    \
    "v_mov_b32_e32 v63, %[iy]\n\t"                                                    \
    "v_mov_b32_e32 v64, %[iz]\n\t"                                                    \
    "s_mov_b32 s62, 0\n\t"                   /* root */                               \
    "s_mov_b32 s63, 0\n\t"                                                            \
    "s_mov_b64 exec, %[live]\n\t"           /* EXEC = the node's active lanes */      \
    "s_mov_b64 %[hits], 0\n\t"                                                        \
    /* ---- record of node s62 from memory (root, pops) ---- */                       \
    ".LBIH_N_%=:\n\t"                        /* s62 = the record's byte offset */      \
    "s_load_dwordx4 s[76:79], %[nodes], s62\n\t"                                      \
    "s_waitcnt lgkmcnt(0)\n\t"                 /* falls into node step A0 */           \
    /* ---- node steps: record buffers A = s[76:83], B = s[36:43] ---- */             \
    BIH_NODE_STEP("A0", CNT_NODE, "s76", "s77", "s78", "s79", "s[36:43]", "s_branch .LBIH_DB_%=\n\t") \
    BIH_NODE_STEP("A1", CNT_NODE, "s80", "s81", "s82", "s83", "s[36:43]", "")          \
    BIH_DESCEND("B", BIH_REC("s36", "s37", "s38", "s39"), BIH_REC("s40", "s41", "s42", "s43"))                                                                  \
    BIH_NODE_STEP("B0", CNT_NODE, "s36", "s37", "s38", "s39", "s[76:83]", "s_branch .LBIH_DA_%=\n\t") \
    BIH_NODE_STEP("B1", CNT_NODE, "s40", "s41", "s42", "s43", "s[76:83]", "")          \
    BIH_DESCEND("A", BIH_REC("s76", "s77", "s78", "s79"), BIH_REC("s80", "s81", "s82", "s83"))                                                                  \
    /* ---- pop until an entry has a searching lane ---- */                           \
    ".LBIH_P_%=:\n\t"                                                                 \
    "s_waitcnt lgkmcnt(0)\n\t"               /* a pair prefetch may be in flight */    \
    ".LBIH_PL_%=:\n\t"                                                                \
    "s_sub_u32 s63, s63, 1\n\t"              /* SCC = borrow: the stack was empty */  \
    "s_cbranch_scc1 .LBIH_X_%=\n\t"                                                   \
    "s_mov_b64 exec, -1\n\t"                                                          \
    "s_cmp_ge_u32 s63, " BIH_S(BIH_ASM_SLOTS) "\n\t"                                  \
    "s_cbranch_scc1 .LBIH_SQ_%=\n\t"                                                  \
    "s_set_gpr_idx_on s63, gpr_idx(SRC0)\n\t"                                         \
    "v_mov_b32_e32 %[tmin], v40\n\t"                                                  \
    "v_mov_b32_e32 %[tmax], v51\n\t"                                                  \
    "s_set_gpr_idx_off\n\t"                                                           \
    ".LBIH_PQ_%=:\n\t"                                                                \
    BIH_POP_NODE(ANY_TEXT)                                                            \
    ".LBIH_SQ_%=:\n\t"                                                              \
    "s_sub_u32 s65, s63, " BIH_S(BIH_ASM_SLOTS) "\n\t"                                \
    "s_lshl_b32 s65, s65, 9\n\t"                                                      \
    "v_add_u32_e32 v35, s65, %[lane4]\n\t"                                            \
    "global_load_dword %[tmin], v35, %[spill]\n\t"                                    \
    "global_load_dword %[tmax], v35, %[spill] offset:256\n\t"                         \
    "s_waitcnt vmcnt(0)\n\t"                                                          \
    "s_branch .LBIH_PQ_%=\n\t"                                                        \
    /* ---- leaves of this node: test them (near first), then descend ---- */         \
    BIH_NODE_LV("A0", "s76", "s77", "s78", "s79")                                     \
    BIH_NODE_LV("A1", "s80", "s81", "s82", "s83")                                     \
    BIH_NODE_LV("B0", "s36", "s37", "s38", "s39")                                     \
    BIH_NODE_LV("B1", "s40", "s41", "s42", "s43")                                     \
    ".LBIH_L_%=:\n\t"                                                                 \
    "s_and_b32 s73, s71, 0x3ffffff\n\t"      /* mid */                                \
    "s_cmp_eq_u32 s72, 0x4000000\n\t"       /* left leaf only */                     \
    "s_cbranch_scc1 .LBIH_L1_%=\n\t"                                                  \
    "s_cmp_eq_u32 s72, 0x80000000\n\t"      /* right leaf only */                    \
    "s_cbranch_scc1 .LBIH_L2_%=\n\t"                                                  \
    "s_mov_b64 s[58:59], s[52:53]\n\t"       /* both children are leaves */           \
    "s_mov_b64 s[60:61], s[54:55]\n\t"                                                \
    "s_bitcmp1_b32 %[near], m0\n\t"                                                   \
    "s_cbranch_scc0 .LBIH_LR_%=\n\t"                                                  \
    BIH_LEAF_L("a", ANY, CNT_LEAF_L, CNT_TRI_L)                                       \
    BIH_LEAF_R("a", ANY, CNT_LEAF_R, CNT_TRI_R)                                       \
    "s_branch .LBIH_P_%=\n\t"                                                         \
    ".LBIH_LR_%=:\n\t"                                                                \
    BIH_LEAF_R("b", ANY, CNT_LEAF_R, CNT_TRI_R)                                       \
    BIH_LEAF_L("b", ANY, CNT_LEAF_L, CNT_TRI_L)                                       \
    "s_branch .LBIH_P_%=\n\t"                                                         \
    ".LBIH_L1_%=:\n\t"                       /* left leaf, right internal */          \
    "s_load_dwordx8 s[76:83], %[nodes], s64\n\t"                                      \
    "s_mov_b64 s[58:59], s[52:53]\n\t"                                                \
    BIH_LEAF_L("c", ANY, CNT_LEAF_L, CNT_TRI_L)                                       \
    CLR("s[54:55]")                                                                   \
    "s_cmp_lg_u64 s[54:55], 0\n\t"                                                    \
    "s_cbranch_scc1 .LBIH_TRA_%=\n\t"                                                 \
    "s_branch .LBIH_P_%=\n\t"                                                         \
    ".LBIH_L2_%=:\n\t"                       /* right leaf, left internal */          \
    "s_load_dwordx8 s[76:83], %[nodes], s64\n\t"                                      \
    "s_mov_b64 s[60:61], s[54:55]\n\t"                                                \
    BIH_LEAF_R("d", ANY, CNT_LEAF_R, CNT_TRI_R)                                       \
    CLR("s[52:53]")                                                                   \
    "s_cmp_lg_u64 s[52:53], 0\n\t"                                                    \
    "s_cbranch_scc1 .LBIH_TLA_%=\n\t"                                                 \
    "s_branch .LBIH_P_%=\n\t"                                                         \
    BIH_PUSH_SPILL("rA", "v32")                                                       \
    BIH_PUSH_SPILL("lA", "v30")                                                       \
    BIH_PUSH_SPILL("rB", "v32")                                                       \
    BIH_PUSH_SPILL("lB", "v30")                                                       \
    ".LBIH_X_%=:\n\t"                                                                 \
    "s_mov_b64 exec, -1\n\t"               /* the statement runs on a full wave */    \
    "s_mov_b32 m0, s70"

#define BIH_PACKET_CLOBBERS                                                           \
    "s36", "s37", "s38", "s39", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47",\
    "s48", "s49", "s50", "s51", "s52", "s53", "s54", "s55", "s56", "s57", "s58", "s59",\
    "s60", "s61", "s62", "s63", "s64", "s65", "s66", "s67", "s68", "s69", "s70", "s71",\
    "s72", "s73", "s76", "s77", "s78", "s79", "s80", "s81", "s82", "s83",           \
    "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", \
    "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", \
    "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", \
    "v60", "v61", "v62", "v63", "v64", BIH_REC_CLOBBERS "vcc", "scc", "memory"
