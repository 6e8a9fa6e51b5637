// pt_bvh_build.cpp — BVH_Build_Iterative (js/BVH_Fast_Builder.js:43-406) as native host code:
// the step before the path. Same tree, same node order, same bits as the
// reference builder, which runs in the page's JavaScript (153 ms for StanfordBunny in Node).
//
// The reference works in JavaScript doubles on float32 inputs (the per-triangle AABB array is a
// Float32Array): box corners are Math.min / Math.max of those inputs (signed zeros as
// ECMAScript defines them), the split value is the double (min + max) * 0.5 of the node's box, and
// centroids are compared to it as doubles. Nodes are emitted depth-first, left subtree first; an
// inner node's right link is filled in when its right child is created. If no axis separates the
// centroids the list is dealt alternately (even positions left).
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/pt.h"

namespace {

// ECMAScript Math.min / Math.max (NaN wins; -0 < +0)
double js_min(double a, double b)
{
    if (a != a || b != b) return NAN;
    if (a == 0.0 && b == 0.0) return std::signbit(a) ? a : b;
    return b < a ? b : a;
}
double js_max(double a, double b)
{
    if (a != a || b != b) return NAN;
    if (a == 0.0 && b == 0.0) return std::signbit(a) ? b : a;
    return a < b ? b : a;
}

struct FlatNode {
    int idObject;       // triangle, or -1 for an inner node
    int idRightChild;   // -1 for a leaf, filled in later for an inner node
    double mn[3], mx[3];
};

struct Builder {
    const float* aabb;  // 9 floats per triangle: min.xyz, max.xyz, centroid.xyz
    std::vector<FlatNode> nodes;
    // the reference's per-depth left / right work lists; `has` = neither null nor undefined
    std::vector<std::vector<uint32_t>> left, right;
    std::vector<char> hasLeft, hasRight;
    int stackptr = 0;

    void ensure(int level)
    {
        if ((int)left.size() <= level) {
            left.resize(level + 1); right.resize(level + 1);
            hasLeft.resize(level + 1, 0); hasRight.resize(level + 1, 0);
        }
    }

    double centroid(uint32_t k, int axis) const { return (double)aabb[9 * (size_t)k + 6 + axis]; }

    // BVH_Create_Node (js/BVH_Fast_Builder.js:43-315)
    void createNode(const std::vector<uint32_t>& work, int idParent, bool isLeftBranch)
    {
        if (work.empty()) return;
        if (work.size() == 1) {
            const uint32_t k = work[0];
            FlatNode leaf;
            leaf.idObject = (int)k;
            leaf.idRightChild = -1;
            for (int a = 0; a < 3; a++) { leaf.mn[a] = aabb[9 * (size_t)k + a]; leaf.mx[a] = aabb[9 * (size_t)k + 3 + a]; }
            const int id = (int)nodes.size();
            nodes.push_back(leaf);
            if (!isLeftBranch) nodes[idParent].idRightChild = id;
            return;
        }
        double mn[3] = { INFINITY, INFINITY, INFINITY }, mx[3] = { -INFINITY, -INFINITY, -INFINITY };
        for (uint32_t k : work)
            for (int a = 0; a < 3; a++) {
                mn[a] = js_min(mn[a], (double)aabb[9 * (size_t)k + a]);
                mx[a] = js_max(mx[a], (double)aabb[9 * (size_t)k + 3 + a]);
            }
        double split[3];
        for (int a = 0; a < 3; a++) split[a] = (mn[a] + mx[a]) * 0.5;   // spatial median
        FlatNode inner;
        inner.idObject = -1;
        inner.idRightChild = 0;
        for (int a = 0; a < 3; a++) { inner.mn[a] = mn[a]; inner.mx[a] = mx[a]; }
        const int id = (int)nodes.size();
        nodes.push_back(inner);
        if (!isLeftBranch) nodes[idParent].idRightChild = id;

        // longest extent first, then the other two (js/BVH_Fast_Builder.js:120-186)
        const double s0 = mx[0] - mn[0], s1 = mx[1] - mn[1], s2 = mx[2] - mn[2];
        int axes[3] = { 0, 1, 2 };
        if (s0 >= s1 && s0 >= s2) { axes[0] = 0; axes[1] = s1 >= s2 ? 1 : 2; axes[2] = s1 >= s2 ? 2 : 1; }
        else if (s1 > s0 && s1 >= s2) { axes[0] = 1; axes[1] = s0 >= s2 ? 0 : 2; axes[2] = s0 >= s2 ? 2 : 0; }
        else if (s2 > s0 && s2 > s1) { axes[0] = 2; axes[1] = s0 >= s1 ? 0 : 1; axes[2] = s0 >= s1 ? 1 : 0; }
        // (no branch taken, e.g. NaN extents: the initial axes 0, 1, 2 stay)

        size_t nl = 0, nr = 0;
        int axis = axes[0];
        for (int j = 0; j < 3; j++) {
            axis = axes[j];
            nl = nr = 0;
            for (uint32_t k : work) (centroid(k, axis) < split[axis] ? nl : nr)++;
            if (nl > 0 && nr > 0) break;
        }
        ensure(stackptr);
        std::vector<uint32_t>& L = left[stackptr];
        std::vector<uint32_t>& R = right[stackptr];
        L.clear(); R.clear();
        if (nl > 0 && nr > 0) {
            L.reserve(nl); R.reserve(nr);
            for (uint32_t k : work) (centroid(k, axis) < split[axis] ? L : R).push_back(k);
        } else {   // no separating axis: deal the list alternately (js/BVH_Fast_Builder.js:281-313)
            for (size_t i = 0; i < work.size(); i++) (i % 2 == 0 ? L : R).push_back(work[i]);
        }
        hasLeft[stackptr] = 1;
        hasRight[stackptr] = 1;
    }

    // BVH_Build_Iterative (js/BVH_Fast_Builder.js:320-380): left branches down, right branches up
    void build(const std::vector<uint32_t>& work)
    {
        nodes.clear();
        nodes.reserve(work.size() * 2);
        std::vector<int> parents;
        stackptr = 0;
        parents.push_back(-1);
        createNode(work, -1, true);
        while (stackptr > -1) {
            ensure(stackptr);
            if (hasLeft[stackptr]) {
                std::vector<uint32_t> cur;
                cur.swap(left[stackptr]);
                hasLeft[stackptr] = 0;
                stackptr++;
                parents.push_back((int)nodes.size() - 1);
                createNode(cur, (int)nodes.size() - 1, true);
            } else if (hasRight[stackptr]) {
                std::vector<uint32_t> cur;
                cur.swap(right[stackptr]);
                hasRight[stackptr] = 0;
                stackptr++;
                const int parent = parents.back();
                parents.pop_back();
                createNode(cur, parent, false);
            } else {
                stackptr--;
            }
        }
    }
};

}  // namespace

extern "C" int pt_bvh_build(const float* aabb_in, const uint32_t* work, int n, float* nodes_out, int max_nodes)
{
    if (!aabb_in || !work || !nodes_out || n < 1) return PT_ERR_ARG;
    Builder b;
    b.aabb = aabb_in;
    b.build(std::vector<uint32_t>(work, work + n));
    if ((int)b.nodes.size() > max_nodes) return PT_ERR_ARG;
    // the texture layout (js/BVH_Fast_Builder.js:384-404): (idObject, min.xyz), (idRightChild, max.xyz)
    for (size_t i = 0; i < b.nodes.size(); i++) {
        const FlatNode& f = b.nodes[i];
        float* o = nodes_out + 8 * i;
        o[0] = (float)f.idObject;
        o[1] = (float)f.mn[0]; o[2] = (float)f.mn[1]; o[3] = (float)f.mn[2];
        o[4] = (float)f.idRightChild;
        o[5] = (float)f.mx[0]; o[6] = (float)f.mx[1]; o[7] = (float)f.mx[2];
    }
    return (int)b.nodes.size();
}
