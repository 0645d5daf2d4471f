/*
 * obj_reader.c -- oracle restatement of the reference OBJ/MTL reader.
 * TEST INFRASTRUCTURE ONLY (see mcpt_oracle.h).
 *
 * Follows CV/Framework/ObjReader.cpp:8-259 and ObjReader.hpp:37-139:
 *  - index 0 of vertices/textures/normals/triangles/materials is a dummy
 *    (ObjReader.hpp:40-54), so 1-based OBJ indices are used unchanged;
 *  - group "default" exists from the start (ObjReader.cpp:17); "g name"
 *    switches group (:51-55); groups are kept in std::map (name) order;
 *  - "usemtl" looks the name up from index 1, 0 if absent (ObjReader.hpp:78-88);
 *  - faces are fan-triangulated: tri k>0 = (v0, prev.v2, vk) (ObjReader.cpp:84-104);
 *  - face vertex forms v, v/t, v//n, v/t/n (ObjReader.hpp:90-138);
 *  - MTL: newmtl reuses an existing name (ObjReader.cpp:196-205); Ka/Kd/Ks
 *    floats, Ks also sets Ns=2 (:225-233); Ns/Tr/Ni doubles (:235-254).
 * orc_model_read_tinyobj restates, independently of the product reader, how
 * QuinEngine loads a scene through tinyobjloader v1.1.1 (tiny_obj_loader.h
 * LoadObj / LoadMtl; QE/Utils/Structure.hpp:9-12, RTX/ShaderResource.hpp:
 * 88-104, 204-215) -- see that function.
 */
#include "oracle_internal.h"

#include <ctype.h>
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static void* xrealloc(void* p, size_t n) {
    void* q = realloc(p, n ? n : 1);
    if (!q) { fprintf(stderr, "oracle: out of memory\n"); abort(); }
    return q;
}

#define PUSH(arr, n, cap, val)                                                \
    do {                                                                      \
        if ((n) == (cap)) {                                                   \
            (cap) = (cap) ? 2 * (cap) : 64;                                   \
            (arr) = xrealloc((arr), (size_t)(cap) * sizeof(*(arr)));          \
        }                                                                     \
        (arr)[(n)++] = (val);                                                 \
    } while (0)

/* ---- a tiny istringstream: whitespace tokens, numeric extraction -------- */
typedef struct {
    const char* p;
    int fail;
} istr;

static void skip_ws(istr* s) {
    while (*s->p && isspace((unsigned char)*s->p)) s->p++;
}

/* operator>>(std::string&): returns 0 on failure (token unchanged) */
static int get_token(istr* s, char* tok, size_t cap) {
    if (s->fail) return 0;
    skip_ws(s);
    if (!*s->p) { s->fail = 1; return 0; }
    size_t n = 0;
    while (*s->p && !isspace((unsigned char)*s->p)) {
        if (n + 1 < cap) tok[n++] = *s->p;
        s->p++;
    }
    tok[n] = 0;
    return 1;
}

/* operator>>(float&) / (double&): value 0 and fail on error */
static double get_number(istr* s, int as_float) {
    if (s->fail) return 0.0;
    skip_ws(s);
    char* end = NULL;
    double v;
    if (as_float) v = (double)strtof(s->p, &end);
    else v = strtod(s->p, &end);
    if (end == s->p) { s->fail = 1; return 0.0; }
    s->p = end;
    return v;
}

/* operator>>(int&) */
static int get_int(istr* s, int* out) {
    if (s->fail) return 0;
    skip_ws(s);
    const char* q = s->p;
    if (*q == '+' || *q == '-') q++;
    if (!isdigit((unsigned char)*q)) { s->fail = 1; *out = 0; return 0; }
    char* end = NULL;
    long v = strtol(s->p, &end, 10);
    s->p = end;
    *out = (int)v;
    return 1;
}

/* operator>>(char&) */
static int get_char(istr* s, char* c) {
    if (s->fail) return 0;
    skip_ws(s);
    if (!*s->p) { s->fail = 1; return 0; }
    *c = *s->p++;
    return 1;
}

/* ObjReader.hpp:90-138 */
static int parse_face_vertex(const char* token, int* v, int* t, int* n) {
    istr b = {token, 0};
    char dummy;
    if (!get_int(&b, v)) return 0;
    if (!get_char(&b, &dummy)) { *t = 0; *n = 0; return 1; }
    if (!get_int(&b, t)) {
        *t = 0;
        b.fail = 0;
        get_char(&b, &dummy);
        if (!get_int(&b, n)) return 0;
        return 1;
    }
    if (!get_char(&b, &dummy)) { *n = 0; return 1; }
    if (!get_int(&b, n)) return 0;
    return 1;
}

static int find_material(const orc_model* m, const char* name) {
    for (int i = 1; i < m->nmats; i++)
        if (strcmp(m->mats[i].name, name) == 0) return i;
    return 0;
}

static int find_add_group(orc_model* m, const char* name) {
    for (int i = 0; i < m->ngroups; i++)
        if (strcmp(m->groups[i].name, name) == 0) return i;
    orc_group g;
    memset(&g, 0, sizeof g);
    g.name = strdup(name);
    PUSH(m->groups, m->ngroups, m->cap_groups, g);
    return m->ngroups - 1;
}

static void mat_init(orc_mat* mt, const char* name) {
    memset(mt, 0, sizeof *mt);
    snprintf(mt->name, sizeof mt->name, "%.*s", (int)sizeof mt->name - 1, name);   /* long names truncated */
    mt->Ns = 1.0; mt->Tr = 0.0; mt->Ni = 1.0;   /* ObjReader.hpp:22 */
}

/* read whole file; returns malloc'd NUL-terminated buffer */
static char* slurp(const char* path) {
    FILE* f = fopen(path, "rb");
    if (!f) return NULL;
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    char* buf = (char*)xrealloc(NULL, (size_t)n + 1);
    size_t r = fread(buf, 1, (size_t)n, f);
    fclose(f);
    buf[r] = 0;
    return buf;
}

/* std::getline with '\\' continuation joining (ObjReader.cpp:23-34) */
typedef struct {
    char* cur;
    char* line;
    size_t cap;
} line_reader;

static int next_line(line_reader* lr) {
    if (!*lr->cur) return 0;
    size_t used = 0;
    for (;;) {
        char* e = strchr(lr->cur, '\n');
        size_t len = e ? (size_t)(e - lr->cur) : strlen(lr->cur);
        if (used + len + 1 > lr->cap) {
            lr->cap = (used + len + 1) * 2;
            lr->line = xrealloc(lr->line, lr->cap);
        }
        memcpy(lr->line + used, lr->cur, len);
        used += len;
        lr->line[used] = 0;
        lr->cur = e ? e + 1 : lr->cur + len;
        if (used > 0 && lr->line[used - 1] == '\\' && *lr->cur) {
            used--;            /* pop_back and append the next line */
            continue;
        }
        return 1;
    }
}

static int read_mtl(orc_model* m, const char* path, char* err, int errlen) {
    char* text = slurp(path);
    if (!text) { snprintf(err, errlen, "Can't open file %s", path); return 0; }
    line_reader lr = {text, NULL, 0};
    int idx = 0;
    char tok[512];
    while (next_line(&lr)) {
        istr s = {lr.line, 0};
        if (!get_token(&s, tok, sizeof tok)) continue;
        if (tok[0] == '#') continue;
        if (!strcmp(tok, "newmtl")) {
            get_token(&s, tok, sizeof tok);
            idx = find_material(m, tok);
            if (idx == 0) {
                orc_mat mt;
                mat_init(&mt, tok);
                PUSH(m->mats, m->nmats, m->cap_mats, mt);
                idx = m->nmats - 1;
            }
        } else if (!strcmp(tok, "Ka") || !strcmp(tok, "Kd") || !strcmp(tok, "Ks")) {
            float x = (float)get_number(&s, 1), y = (float)get_number(&s, 1), z = (float)get_number(&s, 1);
            orc_v3 v = {x, y, z};
            if (tok[1] == 'a') m->mats[idx].Ka = v;
            else if (tok[1] == 'd') m->mats[idx].Kd = v;
            else { m->mats[idx].Ks = v; m->mats[idx].Ns = 2; }
        } else if (!strcmp(tok, "Ns")) {
            m->mats[idx].Ns = get_number(&s, 0);
        } else if (!strcmp(tok, "Tr")) {
            m->mats[idx].Tr = get_number(&s, 0);
        } else if (!strcmp(tok, "Ni")) {
            m->mats[idx].Ni = get_number(&s, 0);
        }
    }
    free(lr.line);
    free(text);
    return 1;
}

static int group_cmp(const void* a, const void* b) {
    return strcmp(((const orc_group*)a)->name, ((const orc_group*)b)->name);
}

int orc_model_read(orc_model* m, const char* path, char* err, int errlen) {
    memset(m, 0, sizeof *m);
    orc_v3 zero = {0, 0, 0};
    PUSH(m->verts, m->nverts, m->cap_verts, zero);
    PUSH(m->normals, m->nnormals, m->cap_normals, zero);
    m->ntexcoords = 1;
    orc_tri t0;
    memset(&t0, 0, sizeof t0);
    PUSH(m->tris, m->ntris, m->cap_tris, t0);
    orc_mat m0;
    mat_init(&m0, "");
    PUSH(m->mats, m->nmats, m->cap_mats, m0);

    char* text = slurp(path);
    if (!text) { snprintf(err, errlen, "Can't open file %s", path); return 0; }
    int grp = find_add_group(m, "default");
    int mat = 0;
    line_reader lr = {text, NULL, 0};
    char tok[512];
    int ok = 1;
    while (ok && next_line(&lr)) {
        istr s = {lr.line, 0};
        if (!get_token(&s, tok, sizeof tok)) continue;
        if (tok[0] == '#') continue;
        if (!strcmp(tok, "mtllib")) {
            get_token(&s, tok, sizeof tok);
            const char* slash = strrchr(path, '/');
            char mpath[4096];
            if (slash) snprintf(mpath, sizeof mpath, "%.*s/%s", (int)(slash - path), path, tok);
            else snprintf(mpath, sizeof mpath, "./%s", tok);
            if (!read_mtl(m, mpath, err, errlen)) ok = 0;
        } else if (!strcmp(tok, "g")) {
            get_token(&s, tok, sizeof tok);   /* on failure tok stays "g" */
            grp = find_add_group(m, tok);
        } else if (!strcmp(tok, "usemtl")) {
            get_token(&s, tok, sizeof tok);
            mat = find_material(m, tok);
        } else if (!strcmp(tok, "f")) {
            int idx = 0;
            orc_tri t;
            memset(&t, 0, sizeof t);
            t.mat = mat;
            PUSH(m->tris, m->ntris, m->cap_tris, t);
            orc_group* g = &m->groups[grp];
            PUSH(g->tris, g->ntris, g->cap, m->ntris - 1);
            while (get_token(&s, tok, sizeof tok)) {
                int vi, ti, ni;
                if (!parse_face_vertex(tok, &vi, &ti, &ni)) {
                    snprintf(err, errlen, "Invalid OBJ file!");
                    ok = 0;
                    break;
                }
                if (idx < 3) {
                    orc_tri* b = &m->tris[m->ntris - 1];
                    b->v[idx] = vi; b->t[idx] = ti; b->n[idx] = ni;
                } else {
                    orc_tri nt;
                    const orc_tri* pv = &m->tris[m->ntris - 1];
                    nt.mat = mat;
                    nt.v[0] = pv->v[0]; nt.v[1] = pv->v[2]; nt.v[2] = vi;
                    nt.t[0] = pv->t[0]; nt.t[1] = pv->t[2]; nt.t[2] = ti;
                    nt.n[0] = pv->n[0]; nt.n[1] = pv->n[2]; nt.n[2] = ni;
                    PUSH(m->tris, m->ntris, m->cap_tris, nt);
                    g = &m->groups[grp];
                    PUSH(g->tris, g->ntris, g->cap, m->ntris - 1);
                }
                ++idx;
            }
        } else if (!strcmp(tok, "v") || !strcmp(tok, "vn")) {
            float x = (float)get_number(&s, 1), y = (float)get_number(&s, 1), z = (float)get_number(&s, 1);
            orc_v3 v = {x, y, z};
            if (tok[1] == 0) PUSH(m->verts, m->nverts, m->cap_verts, v);
            else PUSH(m->normals, m->nnormals, m->cap_normals, v);
        } else if (!strcmp(tok, "vt")) {
            m->ntexcoords++;
        }
    }
    free(lr.line);
    free(text);
    if (!ok) return 0;
    qsort(m->groups, (size_t)m->ngroups, sizeof(orc_group), group_cmp);   /* std::map order */
    return 1;
}

/* ---- tinyobjloader flavor -------------------------------------------------
 * MTL (LoadMtl): every newmtl appends, a lookup finds the first of a name;
 * defaults Ka Kd Ks 0, shininess 1, ior 1, dissolve 1; `d` sets dissolve and
 * wins over `Tr` (dissolve = 1 - Tr); Ks leaves Ns alone; QuinEngine uploads
 * Tr = 1 - dissolve (float).  OBJ (LoadObj): `g` / `o` start a shape, `usemtl`
 * changes the per-face material id within it, fan triangulation (v0, v[k-1],
 * v[k]), negative indices from the end.  Shapes keep file order: each run of
 * one shape's faces with one material becomes a group "%06d:<shape>" (map
 * order = file order), so CreateGeometry sees QuinEngine's triangle order
 * and each triangle's own material.  Material 0 (id -1) is all zero. */
static int read_mtl_tinyobj(orc_model* m, const char* path, char* err, int errlen) {
    char* text = slurp(path);
    if (!text) { snprintf(err, errlen, "Can't open file %s", path); return 0; }
    line_reader lr = {text, NULL, 0};
    int idx = -1, has_d = 0;
    float dissolve = 1.0f;
    char tok[512];
    while (next_line(&lr)) {
        istr s = {lr.line, 0};
        if (!get_token(&s, tok, sizeof tok)) continue;
        if (tok[0] == '#') continue;
        if (!strcmp(tok, "newmtl")) {
            if (idx >= 0) m->mats[idx].Tr = (double)(1.0f - dissolve);
            get_token(&s, tok, sizeof tok);
            orc_mat mt;
            mat_init(&mt, tok);
            mt.Ns = 1.0; mt.Tr = 0.0; mt.Ni = 1.0;
            PUSH(m->mats, m->nmats, m->cap_mats, mt);
            idx = m->nmats - 1;
            has_d = 0;
            dissolve = 1.0f;
            continue;
        }
        if (idx < 0) continue;
        orc_mat* mt = &m->mats[idx];
        if (!strcmp(tok, "Ka") || !strcmp(tok, "Kd") || !strcmp(tok, "Ks")) {
            orc_v3 v;
            v.x = (float)get_number(&s, 0); v.y = (float)get_number(&s, 0); v.z = (float)get_number(&s, 0);
            if (tok[1] == 'a') mt->Ka = v;
            else if (tok[1] == 'd') mt->Kd = v;
            else mt->Ks = v;
        } else if (!strcmp(tok, "Ns")) {
            mt->Ns = (float)get_number(&s, 0);
        } else if (!strcmp(tok, "Ni")) {
            mt->Ni = (float)get_number(&s, 0);
        } else if (!strcmp(tok, "d")) {
            dissolve = (float)get_number(&s, 0);
            has_d = 1;
        } else if (!strcmp(tok, "Tr")) {
            if (!has_d) dissolve = 1.0f - (float)get_number(&s, 0);
        }
    }
    if (idx >= 0) m->mats[idx].Tr = (double)(1.0f - dissolve);
    free(lr.line);
    free(text);
    return 1;
}

int orc_model_read_tinyobj(orc_model* m, const char* path, char* err, int errlen) {
    memset(m, 0, sizeof *m);
    orc_v3 zero = {0, 0, 0};
    PUSH(m->verts, m->nverts, m->cap_verts, zero);
    PUSH(m->normals, m->nnormals, m->cap_normals, zero);
    m->ntexcoords = 1;
    orc_tri t0;
    memset(&t0, 0, sizeof t0);
    PUSH(m->tris, m->ntris, m->cap_tris, t0);
    orc_mat m0;
    memset(&m0, 0, sizeof m0);                 /* all zero, Ns and Ni too */
    PUSH(m->mats, m->nmats, m->cap_mats, m0);

    char* text = slurp(path);
    if (!text) { snprintf(err, errlen, "Can't open file %s", path); return 0; }
    char shape[512] = "";
    int mat = 0, run_mat = -1, runs = 0, grp = -1, fresh = 1;
    line_reader lr = {text, NULL, 0};
    char tok[512];
    int ok = 1;
    int* fv = NULL;
    int nfv = 0, cap_fv = 0;
    while (ok && next_line(&lr)) {
        istr s = {lr.line, 0};
        if (!get_token(&s, tok, sizeof tok)) continue;
        if (tok[0] == '#') continue;
        if (!strcmp(tok, "mtllib")) {
            get_token(&s, tok, sizeof tok);
            const char* slash = strrchr(path, '/');
            char mpath[4096];
            if (slash) snprintf(mpath, sizeof mpath, "%.*s/%s", (int)(slash - path), path, tok);
            else snprintf(mpath, sizeof mpath, "./%s", tok);
            if (!read_mtl_tinyobj(m, mpath, err, errlen)) ok = 0;
        } else if (!strcmp(tok, "g")) {
            if (!get_token(&s, shape, sizeof shape)) shape[0] = 0;
            fresh = 1;
        } else if (!strcmp(tok, "o")) {
            skip_ws(&s);
            snprintf(shape, sizeof shape, "%s", s.p);
            size_t n = strlen(shape);
            while (n && isspace((unsigned char)shape[n - 1])) shape[--n] = 0;
            fresh = 1;
        } else if (!strcmp(tok, "usemtl")) {
            get_token(&s, tok, sizeof tok);
            mat = find_material(m, tok);
        } else if (!strcmp(tok, "f")) {
            if (fresh || mat != run_mat) {
                char key[600];
                snprintf(key, sizeof key, "%06d:%s", runs++, shape);
                grp = find_add_group(m, key);
                run_mat = mat;
                fresh = 0;
            }
            nfv = 0;
            while (get_token(&s, tok, sizeof tok)) {
                int vi, ti, ni;
                if (!parse_face_vertex(tok, &vi, &ti, &ni)) {
                    snprintf(err, errlen, "Invalid OBJ file!");
                    ok = 0;
                    break;
                }
                if (vi < 0) vi += m->nverts;
                if (ti < 0) ti += m->ntexcoords;
                if (ni < 0) ni += m->nnormals;
                PUSH(fv, nfv, cap_fv, vi);
                PUSH(fv, nfv, cap_fv, ti);
                PUSH(fv, nfv, cap_fv, ni);
            }
            for (int k = 2; ok && k < nfv / 3; k++) {
                orc_tri t;
                const int q[3] = {0, k - 1, k};
                for (int j = 0; j < 3; j++) {
                    t.v[j] = fv[3 * q[j]]; t.t[j] = fv[3 * q[j] + 1]; t.n[j] = fv[3 * q[j] + 2];
                }
                t.mat = mat;
                PUSH(m->tris, m->ntris, m->cap_tris, t);
                orc_group* g = &m->groups[grp];
                PUSH(g->tris, g->ntris, g->cap, m->ntris - 1);
            }
        } else if (!strcmp(tok, "v") || !strcmp(tok, "vn")) {
            float x = (float)get_number(&s, 0), y = (float)get_number(&s, 0), z = (float)get_number(&s, 0);
            orc_v3 v = {x, y, z};
            if (tok[1] == 0) PUSH(m->verts, m->nverts, m->cap_verts, v);
            else PUSH(m->normals, m->nnormals, m->cap_normals, v);
        } else if (!strcmp(tok, "vt")) {
            m->ntexcoords++;
        }
    }
    free(fv);
    free(lr.line);
    free(text);
    if (!ok) return 0;
    qsort(m->groups, (size_t)m->ngroups, sizeof(orc_group), group_cmp);   /* "%06d:" keys: file order */
    return 1;
}

void orc_model_free(orc_model* m) {
    for (int i = 0; i < m->ngroups; i++) { free(m->groups[i].name); free(m->groups[i].tris); }
    free(m->groups); free(m->verts); free(m->normals); free(m->tris); free(m->mats);
    memset(m, 0, sizeof *m);
}
