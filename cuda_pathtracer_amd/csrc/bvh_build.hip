// Device build of the reference's SAH BVH (path_tracer/src/BVH_tree.cpp:27-181): the same tree,
// node for node, and the same triangle order as the host restatement (pt_mesh.cpp Builder), so a
// render traverses the tree the reference builds and keeps its first-found tie-break.
//
// The reference's build is a recursion over prim ranges (build_bvh :27-136): union of the range's
// triangle boxes, box of their centres, longest axis, 7-bucket SAH over the centres (its cost loop
// skips bucket i itself and unions the bucket boxes from an all-zero start, boundingbox.h's `||`
// quirk), then libstdc++'s bidirectional std::partition (:121) and the two halves.  On the device:
//   * ranges larger than kSmall prims are processed level by level, one workgroup per range
//     (k_bvh_big): block reductions whose combine keeps the sequential fold's semantics (the first
//     minimum wins ties, so signed zeros match; a box union drops leading all-zero boxes and keeps
//     later ones, as `||` does), the cost loop on one thread, and the partition as the pairs it
//     performs — the i-th misplaced element from the left swapped with the i-th from the right,
//     found by two ordered counts — which is exactly the bidirectional algorithm's result;
//   * ranges of at most kSmall prims are built whole by one thread each (k_bvh_small), in the
//     host recursion's own order;
//   * subtree sizes and inner boxes (left || right) bottom-up, preorder indices top-down (traverse_bvh :138-154: DFS, left child
//     at i + 1), then the flattened nodes and the reordered triangles are written (k_bvh_emit).
// Triangles whose boxes or centres hold a NaN (the fold is then order-dependent in a way the block
// reductions do not reproduce) are handed to the host build (pt::build_bvh_device returns 1) — a
// guard only: the mesh loader rejects non-finite vertices (pt_mesh.cpp append_mesh_impl).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "pt_internal.h"

namespace {

constexpr int kRegions = 7;   // MAX_AREAS - 1 (BVH_tree.cpp:3, :75)
constexpr int kSmall = 128;   // ranges of at most this many prims: one thread builds the subtree
constexpr int kBB = 256;      // threads of k_bvh_big

struct PrimD {   // BVH_BBox (BVH_tree.h): triangle box, its centre, the triangle's load index
    float mn[3], mx[3], c[3];
    int32_t idx;
};
struct BNode {   // a node by creation id: box, children ids (inner) or prim range (leaf)
    float mn[3], mx[3];
    int32_t left, right, axis, start, count;   // count > 0: leaf
    int32_t depth;
    int32_t pad[2];
};
struct Task {
    int32_t start, end, node, depth;
};
struct Ctl {
    uint32_t nodes;       // node ids allocated
    uint32_t nbig;        // big tasks of the next level
    uint32_t nsmall;      // small tasks (built whole by k_bvh_small)
    uint32_t err;         // bits: 1 NaN box, 2 stack, 4 empty range, 8 degenerate split, 16 node capacity
    uint32_t max_depth;
    uint32_t cap;         // node ids available (2n: a binary tree over n >= 1 leaves has 2n - 1)
};

// ---- the reference's box arithmetic (boundingbox.h, as pt_mesh.cpp restates it) ---------------
struct Box {
    float mn[3], mx[3];
};
__device__ __forceinline__ bool is_zero(const Box& b) {
    return b.mn[0] == 0.0f && b.mn[1] == 0.0f && b.mn[2] == 0.0f && b.mx[0] == 0.0f && b.mx[1] == 0.0f &&
           b.mx[2] == 0.0f;
}
__device__ __forceinline__ Box box_union(const Box& self, const Box& o) {   // self || o
    if (is_zero(self)) return o;
    Box r;
    for (int a = 0; a < 3; ++a) {
        r.mn[a] = o.mn[a] < self.mn[a] ? o.mn[a] : self.mn[a];
        r.mx[a] = o.mx[a] > self.mx[a] ? o.mx[a] : self.mx[a];
    }
    return r;
}
__device__ __forceinline__ float box_area(const Box& b) {
    const float dx = b.mx[0] - b.mn[0], dy = b.mx[1] - b.mn[1], dz = b.mx[2] - b.mn[2];
    return 2.0f * ((dx * dy + dx * dz) + dy * dz);
}
__device__ __forceinline__ int longest_axis(const Box& b) {
    const float dx = b.mx[0] - b.mn[0], dy = b.mx[1] - b.mn[1], dz = b.mx[2] - b.mn[2];
    return (dx > dy && dx > dz) ? 0 : (dy > dz) ? 1 : 2;
}
__device__ __forceinline__ int region_of(const Box& cb, const float* c, int axis) {
    float o = c[axis] - cb.mn[axis];   // getOffsetBoxes (boundingbox.h:94-105)
    if (cb.mx[axis] > cb.mn[axis]) o /= (cb.mx[axis] - cb.mn[axis]);
    const float f = kRegions * o;   // (int)(7 o), 7 -> 6; undefined cases clamped as pt_mesh.cpp region_of
    return !(f >= 0.0f) ? 0 : (f >= (float)kRegions ? kRegions - 1 : (int)f);
}
__device__ __forceinline__ Box prim_box(const PrimD& p) {
    Box b;
    for (int a = 0; a < 3; ++a) { b.mn[a] = p.mn[a]; b.mx[a] = p.mx[a]; }
    return b;
}

// A fold of boxes with `||`'s semantics over a contiguous run, combinable in order: the first
// non-zero box starts the union (leading all-zero boxes are dropped), later zero boxes are unioned
// as zeros.  `box` is the union from the first non-zero box; `lead0`: zero boxes before it.
struct UFold {
    Box box;
    int32_t nz;      // a non-zero box seen
    int32_t lead0;   // zero boxes before the first non-zero one
};
__device__ __forceinline__ void ufold_add(UFold& f, const Box& b) {
    if (f.nz) f.box = box_union(f.box, b);
    else if (is_zero(b)) f.lead0 = 1;
    else { f.box = b; f.nz = 1; }
}
__device__ __forceinline__ UFold ufold_cat(const UFold& a, const UFold& b) {   // a's run, then b's
    if (!a.nz) return UFold{b.box, b.nz, (a.lead0 || b.lead0) ? 1 : 0};
    UFold r = a;
    if (b.lead0) r.box = box_union(r.box, Box{{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}});
    if (b.nz) r.box = box_union(r.box, b.box);
    return r;
}
// The fold's result as the reference's accumulated box: the union, or the all-zero box.
__device__ __forceinline__ Box ufold_box(const UFold& f) {
    return f.nz ? f.box : Box{{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};
}
// Centre box (box_union_point from the first centre): min/max keeping the earlier value on ties.
struct CFold {
    Box box;
    int32_t any;
};
__device__ __forceinline__ void cfold_add(CFold& f, const float* p) {
    if (!f.any) {
        for (int a = 0; a < 3; ++a) f.box.mn[a] = f.box.mx[a] = p[a];
        f.any = 1;
        return;
    }
    for (int a = 0; a < 3; ++a) {
        f.box.mn[a] = p[a] < f.box.mn[a] ? p[a] : f.box.mn[a];
        f.box.mx[a] = p[a] > f.box.mx[a] ? p[a] : f.box.mx[a];
    }
}
__device__ __forceinline__ CFold cfold_cat(const CFold& a, const CFold& b) {
    if (!a.any) return b;
    if (!b.any) return a;
    CFold r = a;
    for (int k = 0; k < 3; ++k) {
        r.box.mn[k] = b.box.mn[k] < a.box.mn[k] ? b.box.mn[k] : a.box.mn[k];
        r.box.mx[k] = b.box.mx[k] > a.box.mx[k] ? b.box.mx[k] : a.box.mx[k];
    }
    return r;
}

// Two node ids for the children of a split, or -1 (error bit 16) when the capacity is spent — which
// a partition with both sides non-empty never reaches; the guard keeps a broken split from writing
// past the node array.
__device__ __forceinline__ int alloc_pair(Ctl* ctl) {
    const uint32_t l = atomicAdd(&ctl->nodes, 2u);
    if (l + 2u > ctl->cap) { atomicOr(&ctl->err, 16u); return -1; }
    return (int)l;
}

__device__ void make_leaf(BNode* nodes, int id, const Box& b, int start, int end, int depth, Ctl* ctl) {
    BNode& N = nodes[id];
    N.depth = depth;
    atomicMax(&ctl->max_depth, (uint32_t)depth);
    for (int a = 0; a < 3; ++a) { N.mn[a] = b.mn[a]; N.mx[a] = b.mx[a]; }
    N.left = N.right = -1;
    N.axis = -1;
    N.start = start;
    N.count = end - start;
}
__device__ void make_inner(BNode* nodes, int id, const Box& b, int axis, int l, int r, int start, int depth) {
    BNode& N = nodes[id];
    N.depth = depth;
    for (int a = 0; a < 3; ++a) { N.mn[a] = b.mn[a]; N.mx[a] = b.mx[a]; }
    N.left = l;
    N.right = r;
    N.axis = axis;
    N.start = start;
    N.count = 0;
}

// SAH split of a range from its bucket counts and boxes (BVH_tree.cpp:76-110): the cost loop that
// skips bucket i and unions from the all-zero box, the first minimum.
__device__ __forceinline__ int sah_split(const int* count, const Box* rb, float total_area, float* min_cost) {
    float cost[kRegions - 1];
    for (int i = 0; i < kRegions - 1; ++i) {
        int c0 = 0, c1 = 0;
        Box a0{{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}}, a1{{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};
        for (int j = 0; j < i; ++j) { c0 += count[j]; a0 = box_union(a0, rb[j]); }
        for (int j = i + 1; j < kRegions; ++j) { c1 += count[j]; a1 = box_union(a1, rb[j]); }
        cost[i] = 1.0f * ((float)c0 * box_area(a0) + (float)c1 * box_area(a1)) / total_area;
    }
    float mc = 3.402823466e+38f;   // FLT_MAX
    int split = 0;
    for (int i = 0; i < kRegions - 1; ++i)
        if (cost[i] < mc) { mc = cost[i]; split = i; }
    *min_cost = mc;
    return split;
}

// ---- triangle boxes (Triangle::calculate_boundaries, as pt_mesh.cpp tri_bounds) ----------------
__global__ void k_bvh_prims(const pt_triangle* __restrict__ tris, int n, PrimD* __restrict__ prims, Ctl* ctl) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const pt_triangle& t = tris[i];
        PrimD p;
        bool nan = false;
        for (int a = 0; a < 3; ++a) {
            const float x = t.v[0][a], y = t.v[1][a], z = t.v[2][a];
            const float lo = x < y ? x : y, hi = x > y ? x : y;
            p.mn[a] = lo < z ? lo : z;
            p.mx[a] = hi > z ? hi : z;
            p.c[a] = 0.5f * (p.mn[a] + p.mx[a]);
            nan = nan || p.mn[a] != p.mn[a] || p.mx[a] != p.mx[a] || p.c[a] != p.c[a];
        }
        p.idx = i;
        prims[i] = p;
        if (nan) atomicOr(&ctl->err, 1u);
    }
}

// ---- one level of large ranges, one workgroup per range ----------------------------------------
template <class F, class Cat>
__device__ __forceinline__ F block_cat(F mine, F* s, Cat cat) {   // in thread order, left-biased tree
    const int tid = threadIdx.x;
    s[tid] = mine;
    __syncthreads();
    for (int step = 1; step < kBB; step <<= 1) {
        F v{};
        const bool act = (tid % (2 * step)) == 0;
        if (act) v = cat(s[tid], s[tid + step]);
        __syncthreads();
        if (act) s[tid] = v;
        __syncthreads();
    }
    F r = s[0];
    __syncthreads();
    return r;
}

__global__ __launch_bounds__(kBB) void k_bvh_big(const Task* __restrict__ tasks, int ntasks, PrimD* __restrict__ prims,
                                                 int8_t* __restrict__ region, int32_t* __restrict__ scratch,
                                                 BNode* __restrict__ nodes, Task* __restrict__ next_big,
                                                 Task* __restrict__ small, Ctl* ctl) {
    __shared__ UFold s_u[kBB];
    __shared__ CFold s_c[kBB];
    __shared__ int32_t s_i[kBB];
    __shared__ int32_t s_i2[kBB];
    __shared__ int s_axis, s_split, s_leaf, s_m;
    __shared__ Box s_cb, s_bounds;
    const int tid = threadIdx.x;
    for (int t = blockIdx.x; t < ntasks; t += gridDim.x) {
        const Task T = tasks[t];
        const int n = T.end - T.start;
        const int per = (n + kBB - 1) / kBB;
        const int b0 = T.start + tid * per, b1 = min(b0 + per, T.end);
        // 1. the range's box and its centres' box (build_bvh :34-52)
        UFold u{};
        CFold cf{};
        for (int i = b0; i < b1; ++i) {
            const PrimD p = prims[i];
            ufold_add(u, prim_box(p));
            cfold_add(cf, p.c);
        }
        u = block_cat(u, s_u, ufold_cat);
        cf = block_cat(cf, s_c, cfold_cat);
        if (tid == 0) {
            const Box bounds = ufold_box(u);
            s_bounds = bounds;
            s_cb = cf.box;
            const int axis = longest_axis(cf.box);
            s_axis = axis;
            s_leaf = cf.box.mn[axis] == cf.box.mx[axis];   // all centres equal on it (:53-60)
        }
        __syncthreads();
        const Box cb = s_cb;
        const int axis = s_axis;
        if (s_leaf) {
            if (tid == 0) make_leaf(nodes, T.node, s_bounds, T.start, T.end, T.depth, ctl);
            __syncthreads();
            continue;
        }
        // 2. buckets: count and box per region, in prim order (:75-84)
        for (int i = b0; i < b1; ++i) region[i] = (int8_t)region_of(cb, prims[i].c, axis);
        __shared__ int s_count[kRegions];
        __shared__ Box s_rb[kRegions];
        for (int r = 0; r < kRegions; ++r) {
            UFold f{};
            int c = 0;
            for (int i = b0; i < b1; ++i)
                if (region[i] == r) { ufold_add(f, prim_box(prims[i])); ++c; }
            f = block_cat(f, s_u, ufold_cat);
            s_i[tid] = c;
            __syncthreads();
            if (tid == 0) {
                int tot = 0;
                for (int k = 0; k < kBB; ++k) tot += s_i[k];
                s_count[r] = tot;
                s_rb[r] = ufold_box(f);
            }
            __syncthreads();
        }
        // 3. SAH split on one thread (:86-110); ranges this large never become cost leaves (n > 8)
        if (tid == 0) {
            float mc;
            s_split = sah_split(s_count, s_rb, box_area(s_bounds), &mc);
        }
        __syncthreads();
        const int split = s_split;
        // 4. std::partition (libstdc++ bidirectional, :121): with m = #(region <= split), the k-th
        //    element of [start, start + m) failing the predicate is swapped with the k-th element
        //    of [start + m, end) passing it counted from the right.
        int ntrue = 0;
        for (int i = b0; i < b1; ++i) ntrue += region[i] <= split;
        s_i[tid] = ntrue;
        __syncthreads();
        if (tid == 0) {
            int tot = 0;
            for (int k = 0; k < kBB; ++k) { const int v = s_i[k]; s_i[k] = tot; tot += v; }
            s_m = tot;
        }
        __syncthreads();
        const int m = s_m, mid = T.start + m;
        // falses left of mid (prefix order) and trues right of mid (suffix order)
        int fl = 0, tr = 0;
        for (int i = b0; i < b1; ++i) {
            const bool pr = region[i] <= split;
            fl += (!pr && i < mid);
            tr += (pr && i >= mid);
        }
        s_i[tid] = fl;
        s_i2[tid] = tr;
        __syncthreads();
        if (tid == 0) {
            int a = 0, b = 0;
            for (int k = 0; k < kBB; ++k) {
                const int v = s_i[k], w = s_i2[k];
                s_i[k] = a;
                s_i2[k] = b;
                a += v;
                b += w;
            }
            s_m = b;   // trues right of mid == falses left of mid
        }
        __syncthreads();
        const int ntr = s_m;
        {
            int f = s_i[tid], r = s_i2[tid];
            for (int i = b0; i < b1; ++i) {
                const bool pr = region[i] <= split;
                if (pr && i >= mid) { scratch[T.start + (ntr - 1 - r)] = i; ++r; }   // rank from the right
                (void)f;
            }
        }
        __syncthreads();
        {
            int f = s_i[tid];
            for (int i = b0; i < b1; ++i) {
                const bool pr = region[i] <= split;
                if (!pr && i < mid) {
                    const int j = scratch[T.start + f];
                    const PrimD a = prims[i], b = prims[j];
                    prims[i] = b;
                    prims[j] = a;
                    ++f;
                }
            }
        }
        __syncthreads();
        // 5. the node and its two ranges (:122-128)
        if (tid == 0) {
            const int split_at = (int)(float)mid;
            // both children non-empty (the SAH split always makes them so; a NaN centre box would not,
            // and the level loop would then queue the same range again without end)
            const bool split_ok = split_at > T.start && split_at < T.end;
            if (!split_ok) atomicOr(&ctl->err, 8u);
            const int l = split_ok ? alloc_pair(ctl) : -1;
            if (l >= 0) {
                const int r = l + 1;
                make_inner(nodes, T.node, s_bounds, axis, l, r, T.start, T.depth);
                const Task L{T.start, split_at, l, T.depth + 1}, R{split_at, T.end, r, T.depth + 1};
                if (L.end - L.start > kSmall) next_big[atomicAdd(&ctl->nbig, 1u)] = L;
                else small[atomicAdd(&ctl->nsmall, 1u)] = L;
                if (R.end - R.start > kSmall) next_big[atomicAdd(&ctl->nbig, 1u)] = R;
                else small[atomicAdd(&ctl->nsmall, 1u)] = R;
            }
        }
        __syncthreads();
    }
}

// ---- small ranges: one thread builds the whole subtree, in the host recursion's order ----------
__global__ void k_bvh_small(const Task* __restrict__ tasks, int ntasks, PrimD* __restrict__ prims, BNode* __restrict__ nodes,
                            Ctl* ctl) {
    for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < ntasks; t += gridDim.x * blockDim.x) {
        Task stack[64];
        int top = 0;
        stack[top++] = tasks[t];
        while (top > 0) {
            const Task T = stack[--top];
            const int start = T.start, end = T.end, n = end - start;
            UFold u{};
            for (int i = start; i < end; ++i) ufold_add(u, prim_box(prims[i]));
            // (the reference starts from prims[start]'s box: its union with itself is itself)
            if (n <= 0) { atomicOr(&ctl->err, 4u); continue; }   // (the SAH split never makes one)
            const Box bounds = ufold_box(u);
            if (n == 1) { make_leaf(nodes, T.node, bounds, start, end, T.depth, ctl); continue; }
            CFold cf{};
            for (int i = start; i < end; ++i) cfold_add(cf, prims[i].c);
            const Box cb = cf.box;
            const int axis = longest_axis(cb);
            if (cb.mn[axis] == cb.mx[axis]) { make_leaf(nodes, T.node, bounds, start, end, T.depth, ctl); continue; }
            int mid;
            if (n == 2) {   // nth_element on two elements: swap when the second is smaller
                if (prims[start + 1].c[axis] < prims[start].c[axis]) {
                    const PrimD a = prims[start];
                    prims[start] = prims[start + 1];
                    prims[start + 1] = a;
                }
                mid = (int)(1.0f * (float)(start + end) / 2.0f);
            } else {
                int count[kRegions] = {};
                Box rb[kRegions];
                for (int r = 0; r < kRegions; ++r) rb[r] = Box{{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};
                for (int i = start; i < end; ++i) {
                    const int idx = region_of(cb, prims[i].c, axis);
                    count[idx] += 1;
                    rb[idx] = box_union(rb[idx], prim_box(prims[i]));
                }
                float mc;
                const int split = sah_split(count, rb, box_area(bounds), &mc);
                if (mc >= (float)n && n <= kRegions + 1) { make_leaf(nodes, T.node, bounds, start, end, T.depth, ctl); continue; }
                int first = start, last = end;   // libstdc++ std::partition (bidirectional)
                for (;;) {
                    for (;;) {
                        if (first == last) goto done;
                        if (region_of(cb, prims[first].c, axis) <= split) ++first;
                        else break;
                    }
                    --last;
                    for (;;) {
                        if (first == last) goto done;
                        if (!(region_of(cb, prims[last].c, axis) <= split)) --last;
                        else break;
                    }
                    {
                        const PrimD a = prims[first];
                        prims[first] = prims[last];
                        prims[last] = a;
                    }
                    ++first;
                }
            done:
                mid = (int)(float)first;
            }
            if (top + 2 > 64) { atomicOr(&ctl->err, 2u); break; }
            if (!(mid > start && mid < end)) { atomicOr(&ctl->err, 8u); break; }
            const int l = alloc_pair(ctl), r = l + 1;
            if (l < 0) break;
            make_inner(nodes, T.node, bounds, axis, l, r, start, T.depth);
            stack[top++] = Task{mid, end, r, T.depth + 1};
            stack[top++] = Task{start, mid, l, T.depth + 1};
        }
    }
}

// ---- flatten: subtree sizes bottom-up, preorder indices top-down, one depth per launch --------
// An inner node's box is its children's boxes united, left || right (pt_mesh.cpp Builder::inner),
// not its range's fold: they differ where a child range starts with all-zero boxes, which `||`
// drops from that child but the parent's fold keeps.  Set here, bottom-up, with the sizes.
__global__ void k_bvh_sizes(BNode* __restrict__ nodes, int nnodes, int depth, int32_t* __restrict__ size) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nnodes; i += gridDim.x * blockDim.x) {
        BNode& N = nodes[i];
        if (N.depth != depth) continue;
        if (N.count > 0) { size[i] = 1; continue; }
        size[i] = 1 + size[N.left] + size[N.right];
        Box l, r;
        for (int a = 0; a < 3; ++a) {
            l.mn[a] = nodes[N.left].mn[a]; l.mx[a] = nodes[N.left].mx[a];
            r.mn[a] = nodes[N.right].mn[a]; r.mx[a] = nodes[N.right].mx[a];
        }
        const Box b = box_union(l, r);
        for (int a = 0; a < 3; ++a) { N.mn[a] = b.mn[a]; N.mx[a] = b.mx[a]; }
    }
}
__global__ void k_bvh_preorder(const BNode* __restrict__ nodes, int nnodes, int depth, const int32_t* __restrict__ size,
                               int32_t* __restrict__ pre) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nnodes; i += gridDim.x * blockDim.x) {
        const BNode& N = nodes[i];
        if (N.depth != depth) continue;
        if (depth == 0) pre[i] = 0;   // (the root is node 0)
        if (N.count > 0) continue;    // traverse_bvh: left child at i + 1, right after the left subtree
        const int p = depth == 0 ? 0 : pre[i];
        pre[N.left] = p + 1;
        pre[N.right] = p + 1 + size[N.left];
    }
}
__global__ void k_bvh_emit(const BNode* __restrict__ nodes, int nnodes, const int32_t* __restrict__ pre,
                           pt_bvh_node* __restrict__ out) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nnodes; i += gridDim.x * blockDim.x) {
        const BNode& N = nodes[i];
        pt_bvh_node f;
        for (int a = 0; a < 3; ++a) { f.bmin[a] = N.mn[a]; f.bmax[a] = N.mx[a]; }
        if (N.count > 0) {   // traverse_bvh: leaf (pt_mesh.cpp flatten's field values)
            f.sub_areas = N.count;
            f.first_area_idx = N.start;
            f.axis = -1;
            f.rchild_idx = -1;
        } else {
            f.sub_areas = 0;
            f.axis = N.axis;
            f.first_area_idx = 0;
            f.rchild_idx = pre[N.right];
        }
        out[pre[i]] = f;
    }
}
__global__ void k_bvh_order(const pt_triangle* __restrict__ tris, const PrimD* __restrict__ prims, int n,
                            pt_triangle* __restrict__ out) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) out[i] = tris[prims[i].idx];
}

struct DevBuf {
    std::vector<void*> p;
    ~DevBuf() { for (void* q : p) (void)hipFree(q); }
    template <class T>
    hipError_t get(T** out, size_t n) {
        void* q = nullptr;
        const hipError_t e = hipMalloc(&q, std::max<size_t>(n * sizeof(T), 16));
        if (e == hipSuccess) { p.push_back(q); *out = static_cast<T*>(q); }
        return e;
    }
};

}  // namespace

namespace pt {

// Returns PT_OK (S.bvh / S.triangles filled), 1 (not built on the device: NaN boxes, or more
// nested small ranges than the per-thread stack holds; the caller builds on the host), or an error.
int build_bvh_device(Scene& S, double* ms) {
    S.bvh.clear();
    S.triangles.clear();
    const int n = (int)S.tris_load.size();
    if (n == 0) return PT_OK;
    const auto t0 = std::chrono::steady_clock::now();
    DevBuf B;
    pt_triangle *d_tris = nullptr, *d_out = nullptr;
    PrimD* d_prims = nullptr;
    int8_t* d_region = nullptr;
    int32_t *d_scratch = nullptr, *d_size = nullptr, *d_pre = nullptr;
    BNode* d_nodes = nullptr;
    Task *d_ta = nullptr, *d_tb = nullptr, *d_small = nullptr;
    Ctl* d_ctl = nullptr;
    pt_bvh_node* d_flat = nullptr;
    const size_t max_nodes = 2 * (size_t)n;
    auto hip = [](hipError_t e, const char* w) {
        return e == hipSuccess ? (int)PT_OK : fail(PT_ERR_HIP, std::string("device BVH build: ") + w + ": " + hipGetErrorString(e));
    };
#define BVH_TRY(expr, what) do { if (int rc_ = hip((expr), what)) return rc_; } while (0)
    BVH_TRY(B.get(&d_tris, (size_t)n), "alloc");
    BVH_TRY(B.get(&d_out, (size_t)n), "alloc");
    BVH_TRY(B.get(&d_prims, (size_t)n), "alloc");
    BVH_TRY(B.get(&d_region, (size_t)n), "alloc");
    BVH_TRY(B.get(&d_scratch, (size_t)n), "alloc");
    BVH_TRY(B.get(&d_nodes, max_nodes), "alloc");
    BVH_TRY(B.get(&d_size, max_nodes), "alloc");
    BVH_TRY(B.get(&d_pre, max_nodes), "alloc");
    BVH_TRY(B.get(&d_ta, (size_t)n), "alloc");
    BVH_TRY(B.get(&d_tb, (size_t)n), "alloc");
    BVH_TRY(B.get(&d_small, (size_t)n), "alloc");
    BVH_TRY(B.get(&d_ctl, 1), "alloc");
    BVH_TRY(B.get(&d_flat, max_nodes), "alloc");
    BVH_TRY(hipMemcpy(d_tris, S.tris_load.data(), (size_t)n * sizeof(pt_triangle), hipMemcpyHostToDevice), "upload");
    Ctl c0{1u, 0u, 0u, 0u, 0u, (uint32_t)max_nodes};   // node 0 = the root
    BVH_TRY(hipMemcpy(d_ctl, &c0, sizeof c0, hipMemcpyHostToDevice), "upload");
    const Task root{0, n, 0, 0};
    const int grid = std::min((n + 255) / 256, 2048);
    hipLaunchKernelGGL(k_bvh_prims, dim3(grid), dim3(256), 0, nullptr, d_tris, n, d_prims, d_ctl);
    BVH_TRY(hipGetLastError(), "k_bvh_prims");
    int nbig = 0;
    if (n > kSmall) {
        BVH_TRY(hipMemcpy(d_ta, &root, sizeof root, hipMemcpyHostToDevice), "upload");
        nbig = 1;
    } else {
        BVH_TRY(hipMemcpy(d_small, &root, sizeof root, hipMemcpyHostToDevice), "upload");
        Ctl c1{1u, 0u, 1u, 0u, 0u, (uint32_t)max_nodes};
        BVH_TRY(hipMemcpy(d_ctl, &c1, sizeof c1, hipMemcpyHostToDevice), "upload");
    }
    Task *cur = d_ta, *nxt = d_tb;
    while (nbig > 0) {
        BVH_TRY(hipMemsetAsync(&d_ctl->nbig, 0, sizeof(uint32_t), nullptr), "memset");
        hipLaunchKernelGGL(k_bvh_big, dim3(std::min(nbig, 4096)), dim3(kBB), 0, nullptr, cur, nbig, d_prims, d_region,
                           d_scratch, d_nodes, nxt, d_small, d_ctl);
        BVH_TRY(hipGetLastError(), "k_bvh_big");
        Ctl c;
        BVH_TRY(hipMemcpy(&c, d_ctl, sizeof c, hipMemcpyDeviceToHost), "control read");
        if (c.err) return 1;   // NaN boxes, a degenerate split or the node capacity: the host builds
        nbig = (int)c.nbig;
        std::swap(cur, nxt);
    }
    Ctl c;
    BVH_TRY(hipMemcpy(&c, d_ctl, sizeof c, hipMemcpyDeviceToHost), "control read");
    if (c.nsmall > 0) {
        hipLaunchKernelGGL(k_bvh_small, dim3(std::min(((int)c.nsmall + 63) / 64, 4096)), dim3(64), 0, nullptr, d_small,
                           (int)c.nsmall, d_prims, d_nodes, d_ctl);
        BVH_TRY(hipGetLastError(), "k_bvh_small");
    }
    BVH_TRY(hipMemcpy(&c, d_ctl, sizeof c, hipMemcpyDeviceToHost), "control read");
    if (c.err) return 1;   // NaN boxes or stack: the host builds
    const int nn = (int)c.nodes;
    const int gn = std::min((nn + 255) / 256, 2048);
    for (int dpt = (int)c.max_depth; dpt >= 0; --dpt)
        hipLaunchKernelGGL(k_bvh_sizes, dim3(gn), dim3(256), 0, nullptr, d_nodes, nn, dpt, d_size);
    for (int dpt = 0; dpt <= (int)c.max_depth; ++dpt)
        hipLaunchKernelGGL(k_bvh_preorder, dim3(gn), dim3(256), 0, nullptr, d_nodes, nn, dpt, d_size, d_pre);
    hipLaunchKernelGGL(k_bvh_emit, dim3(std::min((nn + 255) / 256, 2048)), dim3(256), 0, nullptr, d_nodes, nn, d_pre, d_flat);
    hipLaunchKernelGGL(k_bvh_order, dim3(grid), dim3(256), 0, nullptr, d_tris, d_prims, n, d_out);
    BVH_TRY(hipGetLastError(), "flatten");
    S.bvh.resize((size_t)nn);
    S.triangles.resize((size_t)n);
    BVH_TRY(hipMemcpy(S.bvh.data(), d_flat, (size_t)nn * sizeof(pt_bvh_node), hipMemcpyDeviceToHost), "download");
    BVH_TRY(hipMemcpy(S.triangles.data(), d_out, (size_t)n * sizeof(pt_triangle), hipMemcpyDeviceToHost), "download");
#undef BVH_TRY
    if (ms) *ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    S.bvh_built = true;
    return PT_OK;
}

}  // namespace pt
