/* oracle_internal.h -- private structures of the CPU oracle (test infrastructure only). */
#ifndef MCPT_ORACLE_INTERNAL_H
#define MCPT_ORACLE_INTERNAL_H
#include <stdint.h>
#include "mcpt_oracle.h"

typedef struct { float x, y, z; } orc_v3;

typedef struct {            /* ObjReader.hpp:12-18 */
    int v[3], t[3], n[3];
    int mat;
} orc_tri;

typedef struct {            /* ObjReader.hpp:20-30 */
    char name[256];
    orc_v3 Ka, Kd, Ks;
    double Ns, Tr, Ni;
} orc_mat;

typedef struct {            /* ObjReader.hpp:32-35 */
    char* name;
    int* tris;
    int ntris, cap;
} orc_group;

typedef struct {            /* ObjReader.hpp:37-63 */
    orc_v3* verts; int nverts, cap_verts;
    orc_v3* normals; int nnormals, cap_normals;
    int ntexcoords;
    orc_tri* tris; int ntris, cap_tris;
    orc_mat* mats; int nmats, cap_mats;
    orc_group* groups; int ngroups, cap_groups;   /* sorted by name after load */
} orc_model;

typedef struct {            /* Geometry.h:14-35 (pack 1) */
    orc_v3 Ka, Kd, Ks;
    float Ns, Tr, Ni;
    uint32_t start, count;
} orc_geom;

typedef struct {            /* CSKDTree (QE/Utils/Structure.hpp:213-223) without the 64-slot cap */
    uint32_t left, right;
    float bmin[3], bmax[3];
    uint32_t axis;          /* 0 leaf, 1..3 split axis */
    float split;
    uint32_t tri_begin, tri_count;
} orc_node;

struct orc_scene {
    orc_model model;
    orc_geom* geoms; int ngeoms;
    int* tri_geom;          /* per CV triangle: first covering geometry or -1 */
    int* kd_tris; int nkd;  /* kd id -> CV triangle index */
    uint32_t* kd_prio;      /* kd id -> rank in brute-force iteration order (tie-break) */
    orc_node* nodes; int nnodes;
    uint32_t* leaf_ids; int nleaf_ids;
    int kd_depth;
};

int orc_model_read(orc_model* m, const char* path, char* err, int errlen);
int orc_model_read_tinyobj(orc_model* m, const char* path, char* err, int errlen);
void orc_model_free(orc_model* m);
/* KD build over kd triangles (vertex triples), flattened BFS */
void orc_kd_build(orc_scene* s, int kd_build);

#endif
