/*
 * mcpt.h -- C ABI of the MI355X Monte Carlo path-tracing core (libmcpt.so).
 *
 * Drop-in boundary for the reference's tracer module, pw1316/MonteCarloPathTracer
 * CVMCTracer/CVMCTracer/CUDA/CUTracer.h:9-12 (namespace PW::Tracer), whose only
 * caller is CVMCTracer/CVMCTracer/main.cpp:16-18,33-35.  Plain C types only:
 * no HIP, torch or C++ types cross this boundary.  Every function returns
 * MCPT_OK (0) or a negative MCPT_E* code; mcpt_last_error() gives a
 * thread-local message for the last failure on the calling thread.
 *
 *   reference                                         this ABI
 *   ObjModel::readObj(path)  ObjReader.cpp:8-161      mcpt_model_read_obj
 *   cudaError_t Initialize() CUTracer.cu:220-223      mcpt_init
 *   cudaError_t CreateGeometry(const ObjModel*)       mcpt_scene_create (+ KD build,
 *                            CUTracer.cu:225-314       QuinEngine/Utils/KDTree.hpp:58-287)
 *   cudaError_t DestroyGeometry() CUTracer.cu:316-338 mcpt_scene_destroy (frees what it allocated)
 *   cudaError_t RenderScene(int sceneID, PWVector3f*) mcpt_render (host framebuffer, synchronous)
 *                            CUTracer.cu:340-404       mcpt_render_device (device buffer, async)
 *
 * Ownership: a model/scene handle is owned by the caller and used from one
 * thread at a time; the scene owns its device copies; framebuffers are
 * caller-owned.  Framebuffer layout = the reference's hostcolor: row-major
 * y*W + x, linear radiance, fp32 RGB (3 floats per pixel) for mcpt_render;
 * RGBA (4 floats per pixel, A unused) for mcpt_render_device.
 */
#ifndef MCPT_H
#define MCPT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MCPT_ABI_VERSION 9

enum {
    MCPT_OK = 0,
    MCPT_E_INVALID = -1,   /* bad argument                     */
    MCPT_E_IO = -2,        /* file cannot be opened            */
    MCPT_E_PARSE = -3,     /* "Invalid OBJ file!" (ObjReader.cpp:81) */
    MCPT_E_DEVICE = -4,    /* HIP runtime error                */
    MCPT_E_NOMEM = -5,
    MCPT_E_UNSUPPORTED = -6
};

typedef struct mcpt_model mcpt_model;   /* host ObjModel (ObjReader.hpp:37-63)  */
typedef struct mcpt_scene mcpt_scene;   /* device-resident scene + KD tree      */

typedef struct {
    int64_t n_vertices;    /* incl. dummy index 0 (ObjReader.hpp:44) */
    int64_t n_normals;     /* incl. dummy */
    int64_t n_texcoords;   /* incl. dummy */
    int64_t n_triangles;   /* incl. dummy */
    int64_t n_materials;   /* incl. dummy "" material */
    int64_t n_groups;      /* incl. empty ones, std::map order */
} mcpt_model_info;

typedef struct {
    int64_t n_geometries;  /* non-empty groups (CUTracer.cu:278-285) */
    int64_t n_triangles;   /* triangles covered by a geometry range (KD input) */
    int64_t n_nodes;       /* KD nodes, BFS order */
    int64_t n_leaf_refs;   /* total leaf triangle references */
    int64_t kd_depth;      /* deepest node depth (<= 32) */
    int64_t lds_bytes;     /* LDS image size; 0 if the scene is served from global memory */
    int64_t device;        /* HIP device ordinal holding the scene */
    int64_t node_boxes;    /* 1: served from global memory, children culled by their KD boxes */
    int64_t n_devices;     /* devices holding a replica (mcpt_init's list at creation); 0 host-only */
    int64_t kd_build;      /* MCPT_KD_BUILD_* the tree was built with -- ABI 9 */
} mcpt_scene_info;

typedef struct {
    int32_t width, height;      /* full image (IMG_WIDTH/IMG_HEIGHT, CV/stdafx.h:41-42) */
    uint32_t spp;               /* samples per pixel this call (NUM_SAMPLES_PER_KERNEL) */
    uint32_t spp_offset;        /* first global sample index (progressive / sharded spp) */
    uint32_t spp_chunk;         /* samples summed per partial, 0 = spp (summation order) */
    int32_t max_depth;          /* scatter events, reference literal 7 (CUTracer.cu:212) */
    float illum;                /* emitter scale, ILLUM 10 (CV/stdafx.h:45) */
    float fov_deg;              /* horizontal FOV, 60 (CUTracer.cu:189) */
    float eye[3], dir[3], up[3];/* camera lookAt (CUTracer.cu:349-355) */
    uint64_t seed;              /* RNG seed (DESIGN.md determinism spec) */
    uint32_t prev_count;        /* running mean: fb = (fb*prev + mean)/(prev+1) (CUTracer.cu:215-217) */
    int32_t fresnel_kd;         /* 1: Fresnel multiplies Kd (CUTracer.cu:131-133); 0: not (rtx.hlsl:345) */
    int32_t tile;               /* pixel tile edge for sharding/ordering, 0 = 8 */
    int32_t shard_count;        /* tiles t with t % shard_count == shard_index are rendered; 0/1 = all */
    int32_t shard_index;
    int32_t packed;             /* 1: write owned tiles packed (tile-major) instead of row-major */
    int32_t pipeline;           /* MCPT_PIPELINE_*: megakernel (default) or wavefront; same image */
    uint32_t wf_batch;          /* wavefront: max paths per batch and stream (120 B of device memory
                                   each), 0 = automatic: LDS scenes 2^28 on one or two streams,
                                   2^27 on three or more; global-memory scenes 2^28 on one stream,
                                   2^27 on more; a default batch is also capped at work / streams
                                   and shrunk (halved) until the queues fit wf_mem_limit */
    int32_t mode;               /* MCPT_MODE_*: path semantics (default CVMCTracer)       */
    int32_t lean;               /* 1: the megakernel counts only rays (paths, shades, spills,
                                   inner/leaf visits, leaf refs, triangle tests read 0; image and
                                   rays identical; ~1-2% faster); the wavefront's extend drops
                                   its traversal counters (spills, visits, refs, tests read 0;
                                   rays, paths and shades stay).  The counts are deterministic:
                                   a counting render of the same params reports what a lean one
                                   did.  0 (default): count everything */
    int32_t wf_sort;            /* wavefront: 1 = material sort (shade sorts each block of its
                                   queue by material in LDS, so a wave runs one material
                                   branch); 0 (default) = shade in queue order (dense reads,
                                   faster); same image */
    /* Scheduling.  None of these changes the image or the counters, only the
     * time; 0 = automatic (the measured defaults).
     * mcpt_plan_query reports the values a render would use. */
    int32_t wf_streams;         /* wavefront HIP streams 1..4 the batches rotate over; 0: scenes in
                                   LDS 2 (3 for frames of more than 2^29 paths), global-memory scenes 4 */
    int32_t wf_refill;          /* wavefront extend: ready lanes before a wave refills (1..64);
                                   0: 16 (LDS scenes), 8 (global-memory scenes) */
    int32_t wf_group_shift;     /* wavefront, global-memory scenes: paths are dealt to queue
                                   segments in groups of 2^k (6..14); 0: 12 */
    int32_t ready_thresh;       /* megakernel: ready lanes before a shading round (1..64);
                                   0: 32 (LDS scenes), 40 (global-memory scenes) */
    int32_t tail_units_per_lane;/* megakernel tail split: the last units per lane handed out one
                                   sample at a time; 0: 4; < 0: no tail split */
    int32_t tail_units;         /* megakernel: exact number of tail-split units (overrides
                                   tail_units_per_lane when > 0) */
    uint64_t wf_mem_limit;      /* wavefront queue memory per render, bytes; 0: 90% of the device's
                                   free memory (plus what this scene already holds).  A default
                                   batch shrinks to fit; an explicit wf_batch that does not fit
                                   fails with MCPT_E_NOMEM */
    int32_t force_peer_copy;    /* multi-device renders: gather every shard with hipMemcpyPeerAsync,
                                   also between replicas on one device (exercises the cross-device
                                   path on a one-GPU box); 0: peer copies between devices only */
    int32_t gather;             /* multi-device renders (mcpt_init with a device list): how the shards
                                   reach devices[0].  MCPT_GATHER_PEER (0): one hipMemcpyPeerAsync
                                   per device (xGMI DMA).  MCPT_GATHER_RCCL: one ncclGather over a
                                   communicator of the device list (ncclCommInitAll, created on
                                   first use; librccl is loaded then) -- also for a one-device
                                   list, where it is a one-rank gather.  Same image either way */
} mcpt_render_params;

enum {
    MCPT_GATHER_PEER = 0,
    MCPT_GATHER_RCCL = 1
};

enum {
    /* CVMCTracer/CUDA/CUTracer.cu:98-218: 7 scatters + terminal query, ILLUM,
       +-1 px jitter, linear running mean, horizontal fov_deg */
    MCPT_MODE_CVMCTRACER = 0,
    /* MCRT/QuinEngine/Shader/rtx.hlsl:304-405: Russian roulette from bounce
       max_depth, stop at 3*max_depth, no ILLUM, no Fresnel Kd, +-0.5 px jitter,
       near-plane origin, gamma-2.2 running mean, t_best 10000, vertical
       fov_deg, seed = the 32-bit frame seed (GraphicsRTX.cpp:163-193) */
    MCPT_MODE_QUINENGINE = 1
};

enum {
    MCPT_PIPELINE_MEGAKERNEL = 0,   /* one persistent kernel per render (render.hip) */
    MCPT_PIPELINE_WAVEFRONT = 1     /* generate / extend / shade / accumulate queues (wavefront.hip) */
};

typedef struct {
    uint64_t rays;              /* closest-hit queries */
    uint64_t paths;
    uint64_t inner_visits;      /* inner KD nodes visited */
    uint64_t leaf_visits;
    uint64_t leaf_refs;         /* leaf triangle index reads */
    uint64_t tri_tests;
    uint64_t shades;            /* non-terminal hits shaded */
    uint64_t stack_spills;      /* traversal stack entries spilled to global memory */
    uint64_t renders;           /* render calls covered by this record */
    double kernel_ms;           /* summed GPU time of the path kernel */
    double reduce_ms;           /* summed GPU time of the partial-sum reduction */
    int32_t variant;            /* variant of the last call: megakernel 1,2 scene in LDS, 3 global;
                                   wavefront 4 scene in LDS, 5 global */
    int32_t devices;            /* devices the record covers: counters are summed over them,
                                   kernel_ms / reduce_ms are the slowest device's */
} mcpt_render_stats;

/* What a render with given params would run (mcpt_plan_query): the automatic
 * scheduling choices resolved, and the device memory it needs. */
typedef struct {
    int32_t pipeline;           /* MCPT_PIPELINE_* */
    int32_t variant;            /* kernel variant (as mcpt_render_stats::variant) */
    int32_t wf_streams;         /* wavefront streams */
    uint32_t wf_batch;          /* wavefront paths per batch and stream */
    int32_t wf_refill;
    int32_t wf_group_shift;     /* 6 for scenes in LDS (one 8x8 tile per group) */
    int32_t ready_thresh;       /* megakernel */
    int32_t tail_units;         /* megakernel tail-split units */
    uint64_t work_paths;        /* paths of the render (this device's shard) */
    uint64_t workspace_bytes;   /* device memory the render's workspace needs */
    uint64_t wf_queue_bytes;    /* of which the wavefront's queues (what wf_mem_limit bounds) */
    uint64_t device_free_bytes; /* free memory of the scene's device now */
    int32_t devices;            /* devices the render runs on */
    int32_t peer_access;        /* multi-device: 1 if peer access between every pair is enabled */
    uint32_t wf_batch_default;  /* wavefront: the batch the schedule picks with memory unbounded;
                                   wf_batch below it = the queues were shrunk to fit (wf_mem_limit,
                                   the scene's reservation or free device memory) -- ABI 8 */
} mcpt_plan_info;

/* Scene creation options (mcpt_scene_create_ex). */
typedef struct {
    const char* kd_cache_dir;   /* on-disk KD-build cache directory (must exist); NULL = none */
    int32_t host_only;          /* 1: no device allocation */
    int32_t layout;             /* MCPT_LAYOUT_*: scene image placement */
    int32_t kd_build;           /* MCPT_KD_BUILD_*: the KD tree's split rule -- ABI 9 */
} mcpt_scene_options;

enum {
    MCPT_LAYOUT_AUTO = 0,       /* LDS image (8-B nodes) when it fits, else global memory with child boxes */
    MCPT_LAYOUT_GLOBAL = 1      /* global memory with 48-B child-box pair records, whatever the size */
};
/* KD split rule.  Images do not depend on it (the closest hit is the
 * brute-force one for any tree); visit counts and speed do. */
enum {
    MCPT_KD_BUILD_REFERENCE = 0,  /* QuinEngine KDTree.hpp:58-287: median > 64 tris, SAH with Cts = 0 below */
    MCPT_KD_BUILD_SAH = 1         /* SAH with a traversal cost over split-plane regions at every size
                                     (empty space cut off): fewer node visits per ray (host_model.cpp) */
};

/* ---- library ------------------------------------------------------------ */
int mcpt_abi_version(void);
const char* mcpt_last_error(void);
/* Initialize (CUTracer.cu:220-223): select the HIP device(s) used by later
 * scene_create calls on this thread; devices[0] becomes current and holds the
 * scene.  n_devices > 1: the scene is replicated on every listed device, and
 * each unsharded render (shard_count <= 1, packed = 0) is split into
 * n_devices interleaved-tile shards (tile t -> device t % n), rendered
 * concurrently, peer-copied to devices[0] (xGMI DMA) and unpermuted there --
 * the single-device image bit for bit; stats sum the devices.  A device may
 * be listed twice (two replicas on one GPU; RCCL refuses such a list for its
 * gather, mcpt_render_params::gather).  n_devices == 0 keeps the current
 * device and a single-device scene. */
int mcpt_init(const int32_t* devices, int32_t n_devices);
int mcpt_device_count(int32_t* out);
/* fill defaults = the CVMCTracer constants for scene 1 (CUTracer.cu:347-360) */
void mcpt_render_params_default(mcpt_render_params* p);
/* QuinEngine viewer defaults (GraphicsRTX.cpp:163-193, rtx.hlsl:373-404):
 * mode QE, 640x480 (the QE window, QE/Main.cpp:11), 1 spp per frame, depth 5,
 * fovY 45, eye (0,5,17)                                                       */
void mcpt_render_params_quinengine(mcpt_render_params* p);

/* ---- host model (ObjModel) ---------------------------------------------- */
/* In-memory ObjModel, laid out like ObjReader.hpp:57-63 (element 0 of every
 * array is the reference's dummy).  Groups in CSR form, any order (they are
 * re-keyed by name like the reference's std::map).  Arrays are copied.     */
typedef struct {
    const float* vertices;        int64_t n_vertices;    /* 3 floats each  */
    const float* normals;         int64_t n_normals;     /* 3 floats each  */
    const int32_t* triangles;     int64_t n_triangles;   /* 10 ints each: v[3] t[3] n[3] material */
    const double* materials;      int64_t n_materials;   /* 12 doubles each: Ka Kd Ks Ns Tr Ni */
    const char* const* group_names;                      /* n_groups names */
    const int64_t* group_offsets;                        /* n_groups+1 offsets into group_tris */
    const int32_t* group_tris;    int64_t n_groups;
} mcpt_model_desc;
int mcpt_model_create(const mcpt_model_desc* d, mcpt_model** out);
int mcpt_model_read_obj(const char* path, mcpt_model** out);
/* The same with a reader flavor: MCPT_OBJ_CVMCTRACER = mcpt_model_read_obj;
 * MCPT_OBJ_TINYOBJ = what QuinEngine loads through tinyobjloader v1.1.1
 * (QE/Utils/Structure.hpp:9-12, RTX/ShaderResource.hpp:88-104, 204-215):
 * materials with tinyobj's defaults (Ka Kd Ks 0, Ns 1, Ni 1; Tr = 1 - dissolve,
 * `d` wins over `Tr`), shapes in file order, a material per triangle (a group
 * per run of one shape's faces with one material, keyed "%06d:<shape>"). */
int mcpt_model_read_obj_ex(const char* path, int32_t flavor, mcpt_model** out);
enum {
    MCPT_OBJ_CVMCTRACER = 0,    /* CVMCTracer ObjReader (ObjReader.cpp:8-259) */
    MCPT_OBJ_TINYOBJ = 1        /* QuinEngine's tinyobjloader */
};
void mcpt_model_free(mcpt_model* m);
int mcpt_model_get_info(const mcpt_model* m, mcpt_model_info* out);
int mcpt_model_copy_vertices(const mcpt_model* m, float* out);       /* n_vertices*3 */
int mcpt_model_copy_normals(const mcpt_model* m, float* out);        /* n_normals*3 */
int mcpt_model_copy_triangles(const mcpt_model* m, int32_t* out);    /* n_triangles*10: v[3] t[3] n[3] mat */
int mcpt_model_copy_materials(const mcpt_model* m, double* out);     /* n_materials*12: Ka Kd Ks Ns Tr Ni */
/* group g (std::map order): name into buf, triangle count in *n; copy indices if tris != NULL */
int mcpt_model_group(const mcpt_model* m, int64_t g, char* name_buf, int64_t name_cap,
                     int64_t* n, int32_t* tris);

/* ---- scene (CreateGeometry / DestroyGeometry) ---------------------------- */
/* Builds geometries, the KD tree and the device image on the current device.
 * The model is borrowed for the duration of the call only.                 */
int mcpt_scene_create(const mcpt_model* m, mcpt_scene** out);
/* Same, but host-only: no device allocation (KD inspection / CPU tests).   */
int mcpt_scene_create_host(const mcpt_model* m, mcpt_scene** out);
/* Same as mcpt_scene_create (host_only = 0) / _create_host (host_only = 1),
 * with an on-disk KD-build cache in kd_cache_dir (must exist; NULL or "" =
 * no cache).  The tree is a pure function of the triangle vertices, keyed by
 * two 64-bit hashes of them; a file that fails any check is rebuilt and
 * rewritten.  *cache_hit (may be NULL) = 1 if the tree was read, 0 if built.
 * (the reference rebuilds its tree on every start,
 * QuinEngine/RTX/ShaderResource.hpp:128-179.)                              */
int mcpt_scene_create_cached(const mcpt_model* m, const char* kd_cache_dir, int32_t host_only,
                             mcpt_scene** out, int32_t* cache_hit);
/* General form of the three above (options may be NULL = defaults). */
int mcpt_scene_create_ex(const mcpt_model* m, const mcpt_scene_options* options, mcpt_scene** out,
                         int32_t* cache_hit);
void mcpt_scene_destroy(mcpt_scene* s);
int mcpt_scene_get_info(const mcpt_scene* s, mcpt_scene_info* out);
/* KD tree as built (BFS order, QuinEngine/RTX/ShaderResource.hpp:128-179):
 * nodes n_nodes*12 words {left,right,axis(0 leaf,1..3),split bits,min[3],max[3],
 * leaf_begin,leaf_count}; leaf ids = kd triangle ids; kd_tris = kd id -> OBJ
 * triangle index; geoms n_geometries*14 floats {Ka Kd Ks Ns Tr Ni start count} */
int mcpt_scene_copy_kd(const mcpt_scene* s, uint32_t* nodes, uint32_t* leaf_ids,
                       int32_t* kd_tris, float* geoms);

/* ---- render (RenderScene) ------------------------------------------------- */
/* Synchronous; fb_rgb is caller-owned host memory, width*height*3 floats
 * (or, when packed/sharded, owned-pixel-count*3).  Reads fb_rgb when
 * prev_count > 0.  stats may be NULL.                                        */
int mcpt_render(mcpt_scene* s, const mcpt_render_params* p, float* fb_rgb, mcpt_render_stats* stats);
/* Asynchronous on hip_stream (a hipStream_t, NULL = default stream);
 * d_fb_rgba is device memory, 4 floats per output pixel.  Counters and
 * kernel times accumulate until mcpt_render_stats_read(), which waits for
 * the outstanding calls and resets them.                                   */
int mcpt_render_device(mcpt_scene* s, const mcpt_render_params* p, float* d_fb_rgba, void* hip_stream);
int mcpt_render_stats_read(mcpt_scene* s, mcpt_render_stats* out);
/* Diagnostics: synchronous render that also returns, per work unit
 * u = chunk*pixels + pixel, {rays, inner visits, leaf visits, tri tests}
 * (unit_counters: total_units*4 uint32, total_units = pixels * ceil(spp/chunk)). */
int mcpt_render_unit_counters(mcpt_scene* s, const mcpt_render_params* p, float* fb_rgb,
                              uint32_t* unit_counters);
/* number of output pixels a (sharded) render writes, and their (x,y) list */
int64_t mcpt_shard_pixel_count(const mcpt_render_params* p);
int mcpt_shard_pixels(const mcpt_render_params* p, int32_t* xy);      /* count*2 */
/* Closest hit of n caller-given rays on the scene's device, the reference's
 * intersect() (CUTracer.cu:44-96) through the traversal the renders use (the
 * ordered KD walk; scenes in global memory with the child-box cull):
 * o, d = n*3 floats (host); tri_out[i] = kd triangle id (scene_copy_kd's
 * numbering) or -1; hit_out = n*3 floats beta, gamma, t (t = 0 on a miss);
 * t_max = the initial closest t (FLT_MAX in CVMCTracer, 10000 in QuinEngine).
 * stats (may be NULL): rays, inner/leaf visits, leaf refs, tri tests.       */
int mcpt_intersect(mcpt_scene* s, int64_t n, const float* o, const float* d, float t_max,
                   int32_t* tri_out, float* hit_out, mcpt_render_stats* stats);
/* reserve device workspace for p so mcpt_render_device allocates nothing
 * (required before hipGraph capture).  Megakernel workspace per render:
 * partial sums 16 B x pixels x ceil(spp/chunk), the tail-split buffer (16 B
 * per sample of the last ~4 units per lane) and the stack spill area (32 x
 * 16 B per lane); wavefront: 120 B per path of the batch.
 * After a reserve, a render on a CAPTURING stream that needs more than the
 * scene holds fails with MCPT_E_NOMEM before any launch; a render on a
 * non-capturing stream grows the workspace, and the buffers it outgrows are
 * kept (not freed) until mcpt_scene_destroy, so a graph captured earlier
 * stays valid.                                                               */
int mcpt_scene_reserve(mcpt_scene* s, const mcpt_render_params* p);
/* The scheduling a render of p would use and its memory (no allocation, no
 * launch), for a render on a stream that is not capturing a graph (a
 * captured render is held to the scene's reservation, mcpt_scene_reserve).  */
int mcpt_plan_query(mcpt_scene* s, const mcpt_render_params* p, mcpt_plan_info* out);

#ifdef __cplusplus
}
#endif
#endif /* MCPT_H */
