/* price_descent.c -- prices VERDICT r05 item 2 (a speculative replay of a
 * secondary ray's first KD descent along the previous hit's leaf path) on the
 * oracle's exact ordered walk, with no GPU: for every secondary ray of a
 * render, the walk's first-descent inner steps, and how many of them visit
 * the ancestors of the leaf in which the previous ray's hit was accepted
 * (the steps a replay of that ancestor chain would serve from records loaded
 * up front, without a dependent round trip per step).
 *
 * Diagnostic infrastructure only: it compiles the oracle (oracle/render_ref.c,
 * itself test infrastructure) with its ORC_DIAG_* hooks defined.
 *   gcc -O2 -ffp-contract=off -shared -fPIC -o /tmp/price.so scripts/price_descent.c \
 *       oracle/obj_reader.c oracle/kdtree_ref.c -Ioracle -lm -pthread
 * and scripts/price_descent.py drives it.                                    */
#include <stdint.h>
#include <string.h>

#define DIAG_MAXF 96
typedef struct {
    int first_n, first_done;
    uint32_t first[DIAG_MAXF];   /* inner nodes of the walk until its first leaf */
    uint32_t hit_leaf;           /* leaf of the accepted (final) hit, ~0 = miss */
    uint32_t prev_leaf;          /* the previous ray's hit leaf on this path */
} diag_ray;

#define ORC_DIAG_FIELDS diag_ray dg;
#define ORC_DIAG_RAY_BEGIN(q) \
    do { (q)->dg.first_n = 0; (q)->dg.first_done = 0; (q)->dg.hit_leaf = 0xFFFFFFFFu; } while (0)
#define ORC_DIAG_INNER(q, node) \
    do { if (!(q)->dg.first_done && (q)->dg.first_n < DIAG_MAXF) (q)->dg.first[(q)->dg.first_n++] = (node); } while (0)
#define ORC_DIAG_LEAF(q, node) do { (q)->dg.first_done = 1; } while (0)
#define ORC_DIAG_POP(q) do { } while (0)
#define ORC_DIAG_ACCEPT(q, node) do { (q)->dg.hit_leaf = (node); } while (0)
#define ORC_DIAG_AFTER_ISECT(q, depth) diag_after(q, depth)

struct qctx_fwd;
static void diag_after_impl(void* q, int depth);
#define diag_after(q, depth) diag_after_impl((void*)(q), depth)

#include "render_ref.c"

/* parent[] of the BFS node array, chains root -> leaf */
static uint32_t* g_parent;
static int g_nnodes;
static const orc_scene* g_scene;
/* aggregates over secondary rays (single-threaded renders) */
static double g_rays, g_first, g_served, g_inner, g_hist[DIAG_MAXF + 1], g_saved4, g_saved8, g_samechain;

void diag_init(const orc_scene* s) {
    free(g_parent);
    g_scene = s;
    g_nnodes = s->nnodes;
    g_parent = malloc(sizeof(uint32_t) * (size_t)s->nnodes);
    for (int i = 0; i < s->nnodes; i++) g_parent[i] = 0xFFFFFFFFu;
    for (int i = 0; i < s->nnodes; i++)
        if (s->nodes[i].axis) {
            g_parent[s->nodes[i].left] = (uint32_t)i;
            g_parent[s->nodes[i].right] = (uint32_t)i;
        }
    g_rays = g_first = g_served = g_inner = g_saved4 = g_saved8 = g_samechain = 0;
    memset(g_hist, 0, sizeof g_hist);
}

static void diag_after_impl(void* qv, int depth) {
    qctx* q = (qctx*)qv;
    const uint32_t prev = q->dg.prev_leaf;
    q->dg.prev_leaf = q->dg.hit_leaf;
    if (depth == 0 || prev == 0xFFFFFFFFu) return;   /* primary ray, or no previous hit leaf */
    /* ancestors of prev, root first */
    uint32_t chain[DIAG_MAXF];
    int L = 0;
    for (uint32_t n = g_parent[prev]; n != 0xFFFFFFFFu && L < DIAG_MAXF; n = g_parent[n]) chain[L++] = n;
    for (int i = 0; i < L / 2; i++) { uint32_t t = chain[i]; chain[i] = chain[L - 1 - i]; chain[L - 1 - i] = t; }
    const int k = q->dg.first_n;
    int c = 0;
    while (c < k && c < L && q->dg.first[c] == chain[c]) c++;
    g_rays += 1;
    g_first += k;
    g_served += c;
    g_hist[c] += 1;
    if (c == L && k == L) g_samechain += 1;
    /* dependent round trips saved: c serial steps become ceil(c / G) rounds */
    g_saved4 += c - (c + 3) / 4;
    g_saved8 += c - (c + 7) / 8;
    (void)g_nnodes;
}

/* out: rays, first-descent inner steps, served steps, saved (G=4), saved (G=8),
 * rays whose first descent was exactly the previous leaf's chain, hist[0..95] */
void diag_read(double* out) {
    out[0] = g_rays; out[1] = g_first; out[2] = g_served; out[3] = g_saved4; out[4] = g_saved8; out[5] = g_samechain;
    for (int i = 0; i <= DIAG_MAXF; i++) out[6 + i] = g_hist[i];
}
