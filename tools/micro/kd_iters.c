/* Analysis only (not test or product code): per-ray step counts of the reference-mode march under two
 * record layouts, on the oracle's kd-tree (oracle/beam_oracle.c, the reference's tree). Built by
 * tools/kd_iters.py as a separate shared library that includes the oracle's translation unit.
 *   out[4 i + 0]: iterations of the current march (one per visit of a chain of single-child nodes or a
 *                 leaf, hit or miss: k_kd_march_coop's node loop)
 *   out[4 i + 1]: iterations when a node's record holds its children's boxes (only visits whose box is
 *                 hit cost an iteration; the misses are decided in the parent's)
 *   out[4 i + 2]: leaves entered (leaf rounds the lane takes part in)
 *   out[4 i + 3]: deepest stack */
#include "../../oracle/beam_oracle.c"

int32_t exp_kd_iters(const orc_kd* kd, const float* rays, uint32_t n, const float eye[3], const float orient[9],
                     uint32_t* out) {
    for (uint32_t i = 0; i < n; ++i) {
        float dir[3], inv[3];
        orient_dir(dir, orient, rays + (size_t)i * 3);
        for (int c = 0; c < 3; ++c) inv[c] = 1.f / dir[c];
        struct { float mn[3], mx[3]; int32_t node; uint32_t axis; int top; } st[KD_MAX_DEPTH];
        int top = 0, maxtop = 0;
        for (int c = 0; c < 3; ++c) { st[0].mn[c] = kd->wmin; st[0].mx[c] = kd->wmax; }
        st[0].node = 0; st[0].axis = 0; st[0].top = 1; /* top: pushed by a branching node (a chain's first) */
        uint32_t old_it = 0, new_it = 0, leaves = 0;
        float dclosest = FLT_MAX;
        do {
            int chain_top = st[top].top;
            kd_march_entry e; memcpy(e.mn, st[top].mn, 12); memcpy(e.mx, st[top].mx, 12);
            e.node = st[top].node; e.axis = st[top].axis; top--;
            const kd_node* nd = &kd->nodes[e.node];
            if (chain_top) old_it++;
            float box = kd_box_ray(e.mn, e.mx, eye, inv);
            if (box == FLT_MAX) continue;
            int branching = nd->left >= 0 && nd->right >= 0;
            int leaf = nd->left < 0 && nd->right < 0;
            if (branching || leaf) new_it++;
            if (leaf) {
                if (nd->group >= 0) {
                    leaves++;
                    uint32_t cnt = nd->count < KD_LEAF_CAP ? nd->count : KD_LEAF_CAP;
                    const uint32_t* grp = kd->groups + (size_t)nd->group * KD_LEAF_CAP;
                    for (uint32_t k = 0; k < cnt; ++k) {
                        const float* v = kd->s.v + (size_t)grp[k] * 9;
                        float u, vv;
                        float d = tri_intersect(eye, dir, v, v + 3, v + 6, &u, &vv);
                        if (d < dclosest) dclosest = d;
                    }
                    if (dclosest != FLT_MAX) break;
                }
            } else {
                uint32_t a = e.axis, na = (a + 1) % 3;
                float s = .5f * (e.mx[a] + e.mn[a]);
                float p = eye[a] + box * dir[a];
                int order[2] = {p < s ? 1 : 0, p < s ? 0 : 1}; /* pushed first, pushed second (popped first) */
                for (int q = 0; q < 2; ++q) {
                    int right = order[q] == 1;
                    int32_t ch = right ? nd->right : nd->left;
                    if (ch < 0) continue;
                    ++top;
                    memcpy(st[top].mn, e.mn, 12); memcpy(st[top].mx, e.mx, 12);
                    if (right) st[top].mn[a] = s; else st[top].mx[a] = s;
                    st[top].node = ch; st[top].axis = na; st[top].top = branching;
                }
                if (top + 1 > maxtop) maxtop = top + 1;
            }
        } while (top >= 0);
        out[4 * (size_t)i + 0] = old_it;
        out[4 * (size_t)i + 1] = new_it;
        out[4 * (size_t)i + 2] = leaves;
        out[4 * (size_t)i + 3] = (uint32_t)maxtop;
    }
    return 0;
}

/* Per-ray leaf events of the full traversal (no stop at the first hit leaf): ev[MAXE i + k] = the
 * iteration count (old scheme if new_scheme == 0, else the child-box scheme) when the k-th leaf is entered,
 * | 1 << 31 if a face of it is hit, fc[...] its face count; cnt[i] = leaves recorded; tot[i] = iterations of
 * the full traversal. */
int32_t exp_kd_events(const orc_kd* kd, const float* rays, uint32_t n, const float eye[3], const float orient[9],
                      int new_scheme, uint32_t maxe, uint32_t* ev, uint32_t* fc, uint32_t* cnt, uint32_t* tot) {
    for (uint32_t i = 0; i < n; ++i) {
        float dir[3], inv[3];
        orient_dir(dir, orient, rays + (size_t)i * 3);
        for (int c = 0; c < 3; ++c) inv[c] = 1.f / dir[c];
        struct { float mn[3], mx[3]; int32_t node; uint32_t axis; int top; } st[KD_MAX_DEPTH];
        int top = 0;
        for (int c = 0; c < 3; ++c) { st[0].mn[c] = kd->wmin; st[0].mx[c] = kd->wmax; }
        st[0].node = 0; st[0].axis = 0; st[0].top = 1;
        uint32_t it = 0, ne = 0;
        do {
            int chain_top = st[top].top;
            kd_march_entry e; memcpy(e.mn, st[top].mn, 12); memcpy(e.mx, st[top].mx, 12);
            e.node = st[top].node; e.axis = st[top].axis; top--;
            const kd_node* nd = &kd->nodes[e.node];
            if (!new_scheme && chain_top) it++;
            float box = kd_box_ray(e.mn, e.mx, eye, inv);
            if (box == FLT_MAX) continue;
            int branching = nd->left >= 0 && nd->right >= 0;
            int leaf = nd->left < 0 && nd->right < 0;
            if (new_scheme && (branching || leaf)) it++;
            if (leaf) {
                if (nd->group >= 0) {
                    uint32_t c2 = nd->count < KD_LEAF_CAP ? nd->count : KD_LEAF_CAP, hit = 0;
                    const uint32_t* grp = kd->groups + (size_t)nd->group * KD_LEAF_CAP;
                    for (uint32_t k = 0; k < c2; ++k) {
                        const float* v = kd->s.v + (size_t)grp[k] * 9;
                        float u, vv;
                        if (tri_intersect(eye, dir, v, v + 3, v + 6, &u, &vv) < FLT_MAX) hit = 1;
                    }
                    if (ne < maxe) {
                        fc[(size_t)maxe * i + ne] = c2;
                        ev[(size_t)maxe * i + ne++] = it | (hit << 31);
                    }
                }
            } else {
                uint32_t a = e.axis, na = (a + 1) % 3;
                float s = .5f * (e.mx[a] + e.mn[a]);
                float p = eye[a] + box * dir[a];
                int order[2] = {p < s ? 1 : 0, p < s ? 0 : 1};
                for (int q = 0; q < 2; ++q) {
                    int right = order[q] == 1;
                    int32_t ch = right ? nd->right : nd->left;
                    if (ch < 0) continue;
                    ++top;
                    memcpy(st[top].mn, e.mn, 12); memcpy(st[top].mx, e.mx, 12);
                    if (right) st[top].mn[a] = s; else st[top].mx[a] = s;
                    st[top].node = ch; st[top].axis = na; st[top].top = branching;
                }
            }
        } while (top >= 0);
        cnt[i] = ne;
        tot[i] = it;
    }
    return 0;
}
