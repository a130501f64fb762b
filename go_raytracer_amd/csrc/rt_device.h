// rt_device.h — HBM layout of a flattened scene and of the wavefront path state.
// Shared by the host flattener (g++) and the HIP kernels (hipcc).  POD only.
//
// Flattening (host_flatten.cpp) bakes Translate/RotateY (transformation.go) into
// world-space primitives, separates constant media (medium.go) from the
// closest-hit BVH, and turns the lights Hittable (hittable.go:89-103) into a
// weighted table.  See DESIGN.md "Data layout in HBM".
#pragma once
#include <stdint.h>

namespace rt {

struct alignas(16) F4 {
  float x, y, z, w;
};
struct alignas(8) F2 {
  float x, y;
};

// ---- primitive references ------------------------------------------------
// prim ref = (type << 30) | index
enum : uint32_t { PRIM_SPHERE = 0u, PRIM_QUAD = 1u, PRIM_TRI = 2u, PRIM_MEDIUM = 3u };
// Type 3 in a WORLD ref / leaf record is a box leaf (media are never BVH leaves: the
// flattener keeps them apart, so the code is free there).  See "box leaf" below.
constexpr uint32_t PRIM_BOX = 3u;
constexpr uint32_t PRIM_NONE = 0xFFFFFFFFu;
inline constexpr uint32_t prim_ref(uint32_t type, uint32_t idx) { return (type << 30) | idx; }

// ---- BVH2 node: both children's boxes stored in the parent (64 B) --------
//  f4[0] = b0min.xyz | child0 bits      f4[1] = b0max.xyz | child1 bits
//  f4[2] = b1min.xyz | 0                f4[3] = b1max.xyz | 0
// child bits: bit31 set  -> leaf: first ref = (c >> 4) & 0x7FFFFFF, count = (c & 15) + 1
//             bit31 clear-> inner node index
constexpr uint32_t LEAF_BIT = 0x80000000u;
constexpr int MAX_LEAF = 16;
inline constexpr uint32_t leaf_code(uint32_t first, uint32_t count) {
  return LEAF_BIT | (first << 4) | (count - 1u);
}

// ---- BVH4 node: four children's boxes in the parent, SoA (128 B) -----------
//  f4[0] = child codes (bits) of children 0..3   f4[1] = lo.x   f4[2] = hi.x
//  f4[3] = lo.y   f4[4] = hi.y   f4[5] = lo.z   f4[6] = hi.z   f4[7] = 0
//  (codes first: they are fetched with the leaf-record-sized part of a traversal step's
//  loads, so they arrive with the first planes, rt_path.h trav_steps)
// child code: inner BVH4 node index, leaf code (LEAF_BIT, as BVH2), or CHILD_EMPTY
constexpr uint32_t CHILD_EMPTY = 0xFFFFFFFEu;

// ---- BVH8 node: eight children, 16-bit planes relative to the node's box (128 B)
//  f4[0] = origin.xyz | biased exponents (bytes 0-2: plane = origin + q * 2^(E-127))
//  f4[1] = child_base, leaf_base, meta of slots 0-3, meta of slots 4-7
//          meta byte: 0xFF empty; 0x80 | r inner child = node child_base + r;
//          else leaf: records leaf_base + (m & 31), count ((m >> 5) & 3) + 1
//  f4[2..7] = qlo.x, qhi.x, qlo.y, qhi.y, qlo.z, qhi.z (uint16, slot k in halfword k)
// Built by host_bvh8.cpp for scenes of >= kBvh8MinRefs leaf entries.

// ---- per-type primitive records ------------------------------------------
// sphere (objects.go:14-37): sph_cr = center@t0 | radius ; sph_mv = motion | mat bits
//   sph_uv = cos,sin of the baked Y rotation (UV is computed in object space, objects.go:113)
// quad (objects.go:117-140): 5 x F4 = Q|D, u|area, v|mat, n|0, w|0
// triangle (objects.go:242-316): hot 3 x F4 = v0|mat, e0|area, e1|flags
//   attr 6 x F4 = face normal, vn0, vn1, vn2, (uv0,uv1), (uv2,0,0)
enum : uint32_t { TRI_HAS_NORMALS = 1u, TRI_HAS_UV = 2u };

// ---- leaf records: the traversal's copy of each leaf entry (64 B, refs order)
// Built at upload from the per-type arrays; the shading code keeps using those.
//  sphere: Cd = c0.xyz | ref  ;  motion.xyz | r       ; 0 ; 0
//  quad:   Q.xyz | ref        ;  n.xyz | D            ; A = v x w | 0 ; B = w x u | 0
//          (alpha = w.(p x v) = p.A, beta = w.(u x p) = p.B: the triple products of
//           quad.Hit objects.go:186-187 with the cross products hoisted)
//  tri:    v0.xyz | ref       ;  e0.xyz | 0           ; e1.xyz | 0 ; 0
//  box:    C.x C.z ylo | ref  ;  a.x a.z b.x b.z      ; yhi face0 face1 face2 ; face3 face4 face5 0
//          (a NewBox objects.go:208-240 under RotateY/Translate, large scenes only:
//           C = its min corner in world space, a = A / |A|^2 and b = B / |B|^2 for its
//           horizontal edges A (x) and B (z), so x' = (p - C).a and z' = (p - C).b
//           are the box-frame coordinates in [0, 1]; faces are the six quad refs by
//           plane: x' = 0, x' = 1, y = ylo, y = yhi, z' = 0, z' = 1.  One slab test
//           replaces a subtree of six single-quad leaves: rt_kernels.h hit_box_rec)
// Record-loop pair layout (quad-only scenes of <= kBruteMax prims, largest area
// first): records 2p and 2p+1 share 128 B, every field as an adjacent (rec 2p,
// rec 2p+1) float pair so one packed-fp32 op works on both:
//  floats 0-7: nx ny nz D ; 8-13: Qx Qy Qz ; 14-19: Ax Ay Az ; 20-25: Bx By Bz ;
//  26-27: record index (uint bits) ; 28-29: ref ; 30-31: 0.  An odd count is
//  padded with an all-zero record (n = 0: |n.d| < 1e-8, never hit).

// ---- scene features: the fused kernel is instantiated per feature set so that
// code a scene cannot reach (and its register pressure) is compiled out.
// Quads, Lambertian, diffuse lights and solid textures are always supported.
enum : uint32_t {
  FT_SPHERE = 1u, FT_TRI = 2u, FT_METAL = 4u, FT_DIEL = 8u,
  FT_MEDIA = 16u,   // constant media or isotropic materials
  FT_CHECKER = 32u, FT_IMAGE = 64u, FT_NOISE = 128u,
  FT_BOX = 256u,    // box leaves in the world BVH (host_flatten.cpp: large scenes only)
  FT_ALL = 511u
};
// the book2 feature set (C4): spheres, media, textures.  Box leaves are compiled into the
// all-features kernel only: in book2 they measured +-0 (389.5 vs 389.7-391.3 ms at 1024 spp,
// profiles/r4_box_leaves_ab.jsonl) and their box-frame arithmetic moved C4's full-size 8-bit
// parity from 0.9952 to 0.9947, so a book2-like scene keeps its six quads per box
constexpr uint32_t FT_SET_BOOK2 = FT_SPHERE | FT_METAL | FT_DIEL | FT_MEDIA | FT_IMAGE | FT_NOISE;
// Feature sets with a compiled fused kernel, smallest first; a scene runs the first
// set that covers its features (scene_features).
constexpr uint32_t kFtSets[] = {
    0u,                                                     // Cornell box: quads, Lambertian, light
    FT_MEDIA,                                               // + constant media (Cornell smoke)
    FT_SPHERE | FT_TRI | FT_METAL,                          // meshes, spheres, Lambertian + metal
    FT_SPHERE | FT_TRI | FT_METAL | FT_DIEL | FT_CHECKER,   // meshes and spheres, plain materials
    FT_SET_BOOK2,                                           // spheres, media, textures
    FT_ALL};
inline uint32_t pick_ft_set(uint32_t feats) {
  for (uint32_t m : kFtSets)
    if ((feats & ~m) == 0u) return m;
  return FT_ALL;
}

struct DevMedium {           // constantMedium medium.go:13-18
  uint32_t bfirst, bcount;   // boundary prim refs in medium_refs
  float neg_inv_density;     // -1/rho
  int32_t phase_mat;         // isotropic material
  int32_t draw_base;         // first free-flight draw index for this occurrence
  int32_t mult;              // free-flight draws (BVH span-1 leaf duplication, bvh.go:44-46)
  int32_t _pad[2];
};

struct DevLight {            // one leaf of the lights Hittable
  uint32_t ref;              // prim ref, PRIM_NONE for an empty HittableList
  uint32_t lo24;             // pick interval lower bound (24-bit uniform)
  float weight;              // product of 1/len along the list nesting
  float _pad;
};

struct DevMaterial {         // materials.go
  int32_t kind, tex;
  float param;               // metal fuzz / dielectric ior
  float _pad;
  F4 albedo;                 // metal albedo
};

struct DevTexture {          // texture.go
  int32_t kind, a, b, variant;
  F4 color;                  // solid colour; .w = scale (checker inv_scale / noise scale)
};

struct DevImage {
  uint64_t offset;           // into texels
  int32_t w, h;
};

struct DevPerlin {           // perlin.go:10-31
  F4 ranvec[256];
  uint8_t perm[3][256];      // permutations of 0..255, one byte each
};

struct DevScene {
  const F4* sph_cr;
  const F4* sph_mv;
  const F2* sph_uv;
  const F4* quad;
  const F4* tri;
  const F4* tri_attr;
  const F4* nodes;      // the tree this launch traverses (BVH4, or BVH2 for tiny scenes)
  const uint32_t* refs;
  const F4* leafprims;  // 4 x F4 per leaf entry, parallel to refs (see "leaf records")
  const F4* nodes8;     // BVH8 (host_bvh8.cpp layout), root = node 0; null when not built
  const F4* recs8;      // the BVH8's leaf records (leaf record format), in node order
  const F4* big_recs;   // n_big sphere leaf records: radius >= kBigSphereR, not in the BVH
  uint32_t root;
  int32_t n_nodes;
  const DevMedium* media;
  const uint32_t* medium_refs;
  int32_t n_media;
  int32_t medium_draws;
  const DevLight* lights;
  const F4* light_recs;  // 8 F4 per light entry; quad lights: [0..3] the leaf record with the
                         // area in [2].w (pdf), [4..6] Q, u, v (sampling)
  int32_t n_lights;
  int32_t n_refs;       // leaf entries (records)
  const DevMaterial* mats;
  const DevTexture* texs;
  const uint8_t* texels;
  const DevImage* images;
  const DevPerlin* perlins;
  int32_t brute_ax[3];  // record loop (TREE 0): axis-aligned pairs per normal axis, after
                        // the general pairs (host-grouped; rt_path.h brute_axis)
  int32_t brute_vt[3];  // record loop: pairs parallel to an axis (n_a = A_a = 0, B along a:
                        // the sides of boxes rotated about a), between the general and the
                        // axis-aligned pairs (rt_path.h brute_vert; only y is grouped: RotateY
                        // is the reference's only rotation, transformation.go:48)
  int32_t brute_box;    // record loop: pairs of box descriptors after the axis-aligned pairs
                        // (boxes rotated about y, tested as slabs: rt_path.h brute_box),
                        // then the boxes' face records (not looped over)
  int32_t brute_ng;     // record loop: general pairs (the first ones)
  int32_t brute_mx;     // record loop: a mixed pair after the axis-aligned ones, two axis-aligned
                        // records of axes a0 < a1 (rt_path.h brute_mixed): (a0+1) | (a1+1) << 2,
                        // 0 when there is none
  float pdf_floor;      // 1e-30 when every light entry is a prim, else 0 (rt_path.h shade)
  int32_t n_perlins;    // perlin 0's tables are staged in LDS by the noise kernels
  int32_t merge_ok;     // every weight and radiance is >= 0 (solid colours, metal albedos
                        // and, per render, the background): dominated clamp vertices may
                        // be merged (rt_path.h shade_core); else each vertex is pushed
  int32_t shade_lds;    // record-loop kernel of the lean set: F4 offset of the quads' shade
                        // table in the dynamic LDS (after the record pairs), or -1
  int32_t shade_n;      // F4s of that table (2 per quad: normal | kind, solid colour)
  int32_t n_big;        // world spheres tested before the BVH (big_recs, fp64)
};

}  // namespace rt
