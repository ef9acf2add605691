// params.cpp — the reference's tunables and the C-ABI's error strings (host only,
// no device code: also linked into the host-only sanitizer build, tests/san/).
#include "../../include/fccf.h"

extern "C" void fccf_params_default(fccf_params* p) {
  if (!p) return;
  // FCCF.cpp:126-175
  p->parameter_l1 = 0.5f; p->parameter_l2 = 1.0f; p->parameter_k1 = 5.0f; p->parameter_k2 = 2.0f;
  p->normal_vector_threshold1 = 5.0f; p->normal_vector_threshold2 = 8.0f;
  p->face_voxel_size = 1.0f;
  p->voxel_point_threshold = 5;
  p->curvature_threshold = 0.05f;
  p->select_plane_number = 15;
  p->quick_verify_angel_threshold = 10.0f; p->quick_verify_distance_threshold = 2.0f;
  p->required_optimize_plane = 4.0f;
  p->fine_verify_voxel_size = 0.5f; p->fine_verify_number = 4;
  p->included_angle_same_threshold = 5.0f; p->included_angle_min_threshold = 30.0f;
  p->included_angle_max_threshold = 150.0f;
  p->third_plane_threshold = 0.5f; p->third_plane_normal_threshold = 5.0f;
  p->cluster_number_threshold = 10; p->cluster_angel_threshold = 2.0f; p->cluster_distance_threshold = 0.8f;
  p->seclct_cluster_number = 200;
  p->rough_threshold_gl = 2;
}

extern "C" const char* fccf_strerror(int code) {
  switch (code) {
    case FCCF_OK: return "ok";
    case FCCF_E_ARG: return "invalid argument";
    case FCCF_E_HIP: return "HIP runtime error";
    case FCCF_E_RCCL: return "collective error";
    case FCCF_E_OOM: return "out of memory";
    case FCCF_E_IO: return "I/O error";
    case FCCF_E_INTERNAL: return "internal error";
    case FCCF_E_NODEVICE: return "no usable HIP device";
    default: return "unknown error";
  }
}
