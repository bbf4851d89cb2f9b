// rt_host.cpp — host-only scene/header helpers of the C ABI (no GPU calls).
//
//   rt_pack_sphere/plane/rectangle  <- Application::loadShapeBuffer, src/main.cpp:395-469
//   rt_camera_basis                 <- render(), src/main.cpp:772-779
//   rt_set_mode                     <- compute_one_shader header fill, src/main.cpp:584-585
//   rt_fill_rand_buffer             <- fill_rand_buffer, src/main.cpp:535-539 (seeded)
//   rt_moving_light                 <- moving_light, src/main.cpp:541-551
//   rt_init_scene                   <- init_scene1/5/6, src/scene.h:15-167
//   rt_scenegen                     <- synthetic scenes of SURVEY.md §8d
#include <cmath>
#include <cstdint>
#include <cstring>

#include "../../include/rt/abi.h"

namespace {

struct V3 {
  float x, y, z;
};

V3 cross(V3 a, V3 b) { return V3{a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y}; }
// glm::normalize: v * inversesqrt(dot(v, v))
V3 normalize(V3 v) {
  float d = v.x * v.x + v.y * v.y + v.z * v.z;
  float inv = 1.0f / std::sqrt(d);
  return V3{v.x * inv, v.y * inv, v.z * inv};
}

float* shape_ptr(float* header, int i) { return header + rt_off_shapes() / 4 + (size_t)i * 20; }

void set4(float* p, float x, float y, float z, float w) {
  p[0] = x;
  p[1] = y;
  p[2] = z;
  p[3] = w;
}

struct SplitMix64 {
  uint64_t s;
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  // top 24 bits as a float in [0, 1)
  float unit() { return (float)(next() >> 40) * (1.0f / 16777216.0f); }
  float uniform(float a, float b) { return a + (b - a) * unit(); }
};

const V3 kCamLocation{0.0f, 0.0f, 14.0f};  // src/main.cpp:98
const V3 kCamUp{0.0f, 1.0f, 0.0f};         // src/main.cpp:99
const V3 kCamLook{0.0f, 0.0f, 1.0f};       // src/main.cpp:100

void default_header(float* header, int S, int AA, float aspect, int n_objects) {
  std::memset(header, 0, rt_header_bytes(S, AA));
  rt_set_mode(header, 0, n_objects);
  const float loc[3] = {kCamLocation.x, kCamLocation.y, kCamLocation.z};
  const float up[3] = {kCamUp.x, kCamUp.y, kCamUp.z};
  const float look[3] = {kCamLook.x, kCamLook.y, kCamLook.z};
  rt_camera_basis(header, loc, up, look, aspect);
  set4(header + 4 * RT_HDR_LIGHT_POS, -12.0f, 8.0f, 7.0f, 0.0f);  // DEFAULT_LIGHT_POS, main.cpp:47
  // SKY = vec4(13/255.0, 153/255.0, 219/255.0, 0), main.cpp:44
  set4(header + 4 * RT_HDR_BACKGROUND, (float)(13 / 255.0), (float)(153 / 255.0), (float)(219 / 255.0), 0.0f);
}

}  // namespace

extern "C" {

int rt_pack_sphere(float* header, int S, int i, const float c[3], float r, const float color[3],
                   float reflectivity, int emissive) {
  if (!header || !c || !color || i < 0 || i >= S) return RT_E_INVAL;
  float* s = shape_ptr(header, i);
  set4(s + 0, c[0], c[1], c[2], r);                                  // [0] = (center, radius)
  s[4 + 3] = emissive ? 1.0f : 0.0f;                                 // [1].w = emissive
  s[12 + 3] = reflectivity;                                          // [3].w = reflectivity
  set4(s + 16, color[0], color[1], color[2], (float)RT_SHAPE_SPHERE);  // [4] = (color, id)
  return RT_OK;
}

int rt_pack_plane(float* header, int S, int i, const float n[3], float dist, const float color[3],
                  float reflectivity, int emissive) {
  if (!header || !n || !color || i < 0 || i >= S) return RT_E_INVAL;
  float* s = shape_ptr(header, i);
  V3 nn = normalize(V3{n[0], n[1], n[2]});  // member normal = normalize(normal), plane.h:32
  set4(s + 0, nn.x, nn.y, nn.z, dist);
  s[4 + 3] = emissive ? 1.0f : 0.0f;
  // p0 = dist_from_orig * normal, where `normal` is the constructor PARAMETER (plane.h:33)
  set4(s + 12, dist * n[0], dist * n[1], dist * n[2], reflectivity);
  set4(s + 16, color[0], color[1], color[2], (float)RT_SHAPE_PLANE);
  return RT_OK;
}

int rt_pack_rectangle(float* header, int S, int i, const float llc[3], const float right[3],
                      const float up[3], const float color[3], float reflectivity, int emissive) {
  if (!header || !llc || !right || !up || !color || i < 0 || i >= S) return RT_E_INVAL;
  float* s = shape_ptr(header, i);
  V3 n = normalize(cross(V3{right[0], right[1], right[2]}, V3{up[0], up[1], up[2]}));  // rectangle.h:64
  set4(s + 0, n.x, n.y, n.z, 0.0f);
  set4(s + 4, up[0], up[1], up[2], emissive ? 1.0f : 0.0f);
  set4(s + 8, right[0], right[1], right[2], 0.0f);
  set4(s + 12, llc[0], llc[1], llc[2], reflectivity);
  set4(s + 16, color[0], color[1], color[2], (float)RT_SHAPE_RECTANGLE);
  return RT_OK;
}

int rt_camera_basis(float* header, const float location[3], const float up[3], const float look[3],
                    float aspect) {
  if (!header || !location || !up || !look) return RT_E_INVAL;
  V3 w{look[0], look[1], look[2]};
  V3 u = normalize(cross(V3{up[0], up[1], up[2]}, w));
  V3 v = normalize(cross(w, u));
  V3 h{aspect * u.x, aspect * u.y, aspect * u.z};
  // VERT_ASPECT_RATIO (1.0) * v and -0.5 * (...) use main.cpp's operator*(double, vec3)
  V3 vert{(float)(v.x * 1.0), (float)(v.y * 1.0), (float)(v.z * 1.0)};
  V3 hv{h.x + vert.x, h.y + vert.y, h.z + vert.z};
  V3 llc{(float)(hv.x * -0.5) - w.x, (float)(hv.y * -0.5) - w.y, (float)(hv.z * -0.5) - w.z};
  set4(header + 4 * RT_HDR_HORIZONTAL, h.x, h.y, h.z, 0.0f);
  set4(header + 4 * RT_HDR_VERTICAL, vert.x, vert.y, vert.z, 0.0f);
  set4(header + 4 * RT_HDR_LLC_MINUS_CAMPOS, llc.x, llc.y, llc.z, 0.0f);
  set4(header + 4 * RT_HDR_CAMERA_LOCATION, location[0], location[1], location[2], 0.0f);
  return RT_OK;
}

int rt_set_mode(float* header, int frame, int num_objects) {
  if (!header || frame < 0 || num_objects < 0) return RT_E_INVAL;
  header[4 * RT_HDR_MODE + 1] = (float)frame;
  header[4 * RT_HDR_MODE + 2] = (float)num_objects;
  return RT_OK;
}

int rt_fill_rand_buffer(float* header, int S, int AA, uint64_t seed) {
  if (!header || S < 0 || AA <= 0) return RT_E_INVAL;
  SplitMix64 g{seed};
  float* rb = header + rt_off_rand(S) / 4;
  for (int i = 0; i < AA * 2 * 4; ++i) rb[i] = g.unit();
  return RT_OK;
}

int rt_moving_light(float* header, int light_movement) {
  if (!header) return RT_E_INVAL;
  float* L = header + 4 * RT_HDR_LIGHT_POS;
  if (light_movement) {
    for (int k = 0; k < 4; ++k) L[k] = L[k] + 0.1f;  // light_pos + vec4(0.1)
    if (L[0] > 50.0f) set4(L, -50.0f, 20.0f, -50.0f, 0.0f);
  } else {
    set4(L, -12.0f, 8.0f, 7.0f, 0.0f);
  }
  return RT_OK;
}

int rt_scenegen(float* header, int S, int n_objects, int AA, uint64_t seed, float aspect) {
  if (!header || S < 0 || n_objects < 0 || n_objects > S || AA <= 0) return RT_E_INVAL;
  default_header(header, S, AA, aspect, n_objects);
  SplitMix64 g{seed};
  for (int i = 0; i < n_objects; ++i) {
    if (i == 0) {  // ground, as scene5/6 (src/scene.h:96-99)
      const float c[3] = {0.0f, -35.0f, 0.0f}, col[3] = {0.8f, 0.6f, 0.2f};
      rt_pack_sphere(header, S, 0, c, 33.0f, col, 1.0f, 0);
      continue;
    }
    float c[3] = {g.uniform(-12.0f, 12.0f), g.uniform(-2.0f, 6.0f), g.uniform(-20.0f, 4.0f)};
    float r = g.uniform(0.3f, 1.5f);
    float col[3] = {g.uniform(0.1f, 0.9f), g.uniform(0.1f, 0.9f), g.uniform(0.1f, 0.9f)};
    float p_refl = g.unit(), refl_v = g.uniform(0.0f, 0.6f), p_emis = g.unit();
    float refl = p_refl < 0.6f ? 1.0f : refl_v;
    int emissive = p_emis < (1.0f / 16.0f);
    if (emissive)
      for (float& k : col) k *= 4.0f;
    rt_pack_sphere(header, S, i, c, r, col, refl, emissive);
  }
  return rt_fill_rand_buffer(header, S, AA, 7000);
}

int rt_init_scene(float* header, int S, int AA, int which, float aspect) {
  if (!header || AA <= 0) return RT_E_INVAL;
  struct Sph {
    float c[3], r, col[3], refl;
    int emis;
  };
  if (which == 1) {  // src/scene.h:15-65
    if (S < 5) return RT_E_INVAL;
    default_header(header, S, AA, aspect, 5);
    const Sph sp[4] = {{{0, -0.5f, 0}, 2, {0.8f, 0.2f, 0.5f}, 0.5f, 0},
                       {{4, -0.5f, -2}, 3.5f, {0.8f, 0.8f, 0.1f}, 0.9f, 0},
                       {{-4.5f, 4, -15}, 4, {0.2f, 0.8f, 0.1f}, 0.2f, 0},
                       {{-8, -1, 2}, 1.5f, {1, 1, 1}, 0.0f, 0}};
    for (int i = 0; i < 4; ++i) rt_pack_sphere(header, S, i, sp[i].c, sp[i].r, sp[i].col, sp[i].refl, sp[i].emis);
    const float n[3] = {0, 1, 0}, col[3] = {0.3f, 0.0f, 0.5f};
    rt_pack_plane(header, S, 4, n, -4.0f, col, 1.0f, 0);
  } else if (which == 5) {  // src/scene.h:67-109
    if (S < 3) return RT_E_INVAL;
    default_header(header, S, AA, aspect, 3);
    const Sph sp[3] = {{{0, 18, 0}, 10, {1.5f, 1.5f, 1.5f}, 1.0f, 1},
                       {{0, 0, 0}, 2, {0.2f, 0.6f, 0.8f}, 0.4f, 0},
                       {{0, -35, 0}, 33, {0.8f, 0.6f, 0.2f}, 1.0f, 0}};
    for (int i = 0; i < 3; ++i) rt_pack_sphere(header, S, i, sp[i].c, sp[i].r, sp[i].col, sp[i].refl, sp[i].emis);
  } else if (which == 6) {  // src/scene.h:111-167
    if (S < 6) return RT_E_INVAL;
    default_header(header, S, AA, aspect, 6);
    const Sph sp[6] = {{{0, 12, 0}, 6, {4, 4, 4}, 1.0f, 1},
                       {{-8, 0, 0}, 2, {8, 8, 16}, 1.0f, 1},
                       {{0, 0, 0}, 2, {0.2f, 0.6f, 0.8f}, 0.4f, 0},
                       {{0, -35, 0}, 33, {0.8f, 0.6f, 0.2f}, 1.0f, 0},
                       {{2, 1, 3}, 0.5f, {1, 1, 1}, 0.0f, 0},
                       {{4.5f, 0.2f, 5}, 2.25f, {1, 1, 1}, 0.0f, 0}};
    for (int i = 0; i < 6; ++i) rt_pack_sphere(header, S, i, sp[i].c, sp[i].r, sp[i].col, sp[i].refl, sp[i].emis);
  } else {
    return RT_E_INVAL;
  }
  return rt_fill_rand_buffer(header, S, AA, 7000);
}

}  // extern "C"
