// geom.hip — tracking + geometry stages (see vo_geom.h).
#include "vo_geom.h"
#include <cstring>

namespace vo {

hipError_t geom_alloc(GeomBuffers& g, int max_frames, int kp_cap, int n_hyp)
{
    g.max_frames = max_frames; g.kp_cap = kp_cap; g.n_hyp = n_hyp;
    const size_t F = max_frames, K = kp_cap;
    hipError_t e;
#define GA(ptr, bytes) do { e = hipMalloc((void**)&(ptr), (bytes)); if (e != hipSuccess) return e; } while (0)
    GA(g.lists, sizeof(int) * F * TL_COUNT * K);
    GA(g.list_n, sizeof(int) * F * 4);
    GA(g.step_i, sizeof(int) * 4 * F * K);
    GA(g.step_j, sizeof(int) * 4 * F * K);
    GA(g.step_n, sizeof(int) * 4 * F);
    GA(g.world, sizeof(double) * F * K * 3);
    GA(g.imgpt, sizeof(double) * F * K * 2);
    GA(g.oldpos, sizeof(float) * F * K * 4);
    GA(g.inliers, F * K);
    GA(g.hyp, sizeof(MsacHyp) * F * n_hyp);
    GA(g.fg, sizeof(FrameGeom) * F);
    GA(g.lm_new, sizeof(int) * F * K);
    GA(g.lm_M, sizeof(int) * F);
    GA(g.lm_X, sizeof(float) * F * K * 3);
    GA(g.lm_keep, F * K);
    GA(g.lm_rows, sizeof(int) * F);
#undef GA
    return hipSuccess;
}

void geom_free(GeomBuffers& g)
{
    hipFree(g.lists); hipFree(g.list_n); hipFree(g.step_i); hipFree(g.step_j); hipFree(g.step_n); hipFree(g.world);
    hipFree(g.imgpt); hipFree(g.oldpos); hipFree(g.inliers); hipFree(g.hyp); hipFree(g.fg); hipFree(g.lm_new);
    hipFree(g.lm_M); hipFree(g.lm_X); hipFree(g.lm_keep); hipFree(g.lm_rows);
    g = GeomBuffers();
}

void geom_fill_track_jobs(const GeomBuffers& g, MatchJob* jobs, int max_frames, int first, const SiftBuffers& sb,
                          int* pair_i, int* pair_j, int* pair_n, int kp_cap)
{
    (void)g; (void)jobs; (void)max_frames; (void)first; (void)sb; (void)pair_i; (void)pair_j; (void)pair_n; (void)kp_cap;
}

}  // namespace vo
