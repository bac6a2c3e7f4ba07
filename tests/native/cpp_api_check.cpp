// C++ host-side check of include/sfrt.hpp, written the way the reference drives
// its renderers (paths under /root/reference/Raytracing/):
//  * SphereWorld: the constructor's scene (SphereWorld.cpp:58-62: AddSphere of
//    {0,0,0,4} then 10 rand() spheres after srand(0), arguments evaluated right
//    to left as g++ does), width/height set like Source.cpp:40-41, and the frame
//    filled by 8 threads x 4 column cycles exactly as RenderThread does
//    (Source.cpp:17-28) -- then compared with the golden hash of that frame;
//  * Shader: the uniform uploads of every UpdateSpheres call the constructor
//    makes (SphereWorld.cpp:214-238), main()'s camera uniforms
//    (Source.cpp:143-146) and one draw -- compared with the GLSL golden hash.
// Built and run by tests/test_gpu_parity.py::test_cpp_host_api.
//   cpp_api_check <assets dir> <sphere 1080p fnv1a64> <glsl 320x180 fnv1a64>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <string>
#include <thread>
#include <vector>

#include "sfrt.hpp"

namespace {

std::string fnv1a64(const std::vector<uint8_t>& b) {
  uint64_t h = 0xcbf29ce484222325ULL;
  for (uint8_t c : b) {
    h ^= c;
    h *= 0x100000001b3ULL;
  }
  char s[17];
  std::snprintf(s, sizeof s, "%016llx", (unsigned long long)h);
  return s;
}

sfrt::Image load_raw(const std::string& path, int w, int h) {
  sfrt::Image img;
  img.pixels.resize((size_t)w * h * 4);
  std::ifstream f(path, std::ios::binary);
  f.read(reinterpret_cast<char*>(img.pixels.data()), (std::streamsize)img.pixels.size());
  if (!f) throw std::runtime_error("cannot read " + path);
  img.width = w;
  img.height = h;
  return img;
}

struct Ball {  // struct Sphere (SphereWorld.h:23-29), the fields the uploads read
  sfrt::Vector3f pos;
  float radius;
  sfrt::Vec4 light;
};

}  // namespace

int main(int argc, char** argv) {
  if (argc < 4) return 2;
  const std::string assets = argv[1];
  int failures = 0;
  try {
    const sfrt::Image floor = load_raw(assets + "/floor_128x128.rgba", 128, 128);

    // ---- SphereWorld::SphereWorld (SphereWorld.cpp:43-74), frame fill part ----
    sfrt::SphereWorld world(0);
    sfrt::Shader shader(0);
    world.LoadTexture(floor);
    shader.setGround(floor);
    std::vector<Ball> lights, ospheres;
    // SphereWorld::UpdateSpheres (SphereWorld.cpp:199-238) after each Add*
    auto update_spheres = [&]() {
      world.UpdateSpheres();
      const std::vector<sfrt_sphere> s = world.Spheres();
      const int ns = (int)s.size(), nl = (int)lights.size();
      for (int i = 0; i < ns; i++) {
        shader.setUniform("spheres[" + std::to_string(i) + "]",
                          sfrt::Vec4{s[i].x, s[i].y, s[i].z, s[i].radius});
        shader.setUniform("lights[" + std::to_string(i) + "]", sfrt::Vec4{0, 0, 0, 0});
        shader.setUniform("uvs[" + std::to_string(i) + "]", sfrt::Vec4{0.5f, 0.0f, 0, 0});
      }
      for (int i = 0; i < nl; i++) {
        const Ball& L = lights[i];
        shader.setUniform("spheres[" + std::to_string(i + ns) + "]",
                          sfrt::Vec4{L.pos.x, L.pos.y, L.pos.z, L.radius});
        shader.setUniform("lights[" + std::to_string(i + ns) + "]",
                          sfrt::Vec4{L.light.x, L.light.y, L.light.z, 1});
      }
      for (int i = 0; i < (int)ospheres.size(); i++) {
        const Ball& O = ospheres[i];
        shader.setUniform("spheres[" + std::to_string(i + ns + nl) + "]",
                          sfrt::Vec4{O.pos.x, O.pos.y, O.pos.z, O.radius});
        shader.setUniform("lights[" + std::to_string(i + ns + nl) + "]", O.light);
        shader.setUniform("uvs[" + std::to_string(i + ns + nl) + "]",
                          sfrt::Vec4{0.5f, 1.0f, 0.5f, 0.0f});
      }
      shader.setUniform("lightCount", nl);
      shader.setUniform("sphereCount", ns);
      shader.setUniform("allSpheresCount", nl + ns + (int)ospheres.size());
    };
    auto add_light = [&](sfrt::Vector3f pos, float radius, sfrt::Vec4 color, bool notlight) {
      (notlight ? ospheres : lights).push_back(Ball{pos, radius, color});
      update_spheres();
    };
    std::srand(0);
    world.AddSphere({0, 0, 0}, 4);
    update_spheres();
    for (int i = 0; i < 10; i++) {
      const float r = (float)(std::rand() % 6 + 2);   // right-to-left argument evaluation
      const float z = (float)(std::rand() % 20 - 10);
      const float y = (float)(std::rand() % 10 - 5);
      const float x = (float)(std::rand() % 20 - 10);
      world.AddSphere({x, y, z}, r);
      update_spheres();
    }
    for (int i = 0; i < 10; i++) {
      const float r = (float)(std::rand() % 2 + 1) * 0.3f;
      add_light({(float)i * 1.2f, 1, 1}, r, sfrt::Vec4{0.5f, 1, 1, 1}, true);
    }
    add_light({0, -1, 1}, 0.2f, sfrt::Vec4{1, 1, 1, 1}, false);

    // ---- main(): world.width/height (Source.cpp:40-41), RenderThread x 8 ----
    world.width = 1920;
    world.height = 1080;
    const int threadCount = 8, fullCycles = 4;
    std::vector<uint8_t> frame((size_t)world.width * world.height * 4, 0);
    std::vector<std::thread> threads;
    for (int num = 0; num < threadCount; num++)
      threads.emplace_back([&, num]() {
        short cycle = 0;
        for (int k = 0; k < fullCycles; k++) {   // one full frame = fullCycles draws
          world.UpdateImage(frame.data(), (short)num, (short)threadCount, cycle, (short)fullCycles);
          cycle = (short)((cycle + 3) % fullCycles);
        }
      });
    for (auto& t : threads) t.join();
    const std::string hs = fnv1a64(frame);
    std::printf("sphereworld 1920x1080 interleaved fnv1a64=%s want=%s\n", hs.c_str(), argv[2]);
    if (hs != argv[2]) failures++;
    std::vector<uint8_t> whole(frame.size(), 0);
    world.UpdateImage(whole.data(), 0, 1, 0, 1);
    if (whole != frame) {
      std::printf("single-call frame differs from the interleaved one\n");
      failures++;
    }

    // ---- the same frame on several GPUs: devices {0, 0} (peer copies) and {0} (RCCL),
    //      bands packed (the default for Floor.png's 0/255 alphas) and RGBA8 ----
    for (const std::vector<int>& devs : {std::vector<int>{0, 0}, std::vector<int>{0}}) {
      for (int fmt : {SFRT_TRANSFER_AUTO, SFRT_TRANSFER_RGBA}) {
        sfrt::MultiSphereWorld multi(devs);
        multi.LoadTexture(floor);
        multi.SetSpheres(world.Spheres());
        multi.SetTransfer(fmt);
        multi.width = world.width;
        multi.height = world.height;
        multi.cam = world.cam;
        std::vector<uint8_t> mf(frame.size(), 0);
        multi.UpdateImage(mf.data());
        const std::string hm = fnv1a64(mf);
        std::printf("multi x%zu transfer %d 1920x1080 fnv1a64=%s want=%s\n", devs.size(), fmt,
                    hm.c_str(), argv[2]);
        if (hm != argv[2]) failures++;
      }
    }

    // ---- main(): shader uniforms and rt.draw (Source.cpp:143-153) at 320x180 ----
    const int W = 320, H = 180;
    shader.setUniform("campos", world.cam.pos);
    shader.setUniform("rotation", sfrt::Vector2f{world.cam.rotation, world.cam.hrotation});
    shader.setUniform("fov", sfrt::Vector2f{world.cam.fovH, world.cam.fovV});
    shader.setUniform("size", sfrt::Vector2f{(float)W, (float)H});
    std::vector<uint8_t> rt((size_t)W * H * 4);
    shader.drawImage(rt.data(), W, H);
    const std::string hg = fnv1a64(rt);
    std::printf("shader 320x180 fnv1a64=%s want=%s\n", hg.c_str(), argv[3]);
    if (hg != argv[3]) failures++;

    // ---- errors surface as sfrt::Error with the C ABI code ----
    try {
      shader.setUniform("nosuch", 1.0f);
      failures++;
    } catch (const sfrt::Error& e) {
      if (e.code() != SFRT_E_INVALID) failures++;
    }
  } catch (const std::exception& e) {
    std::printf("exception: %s\n", e.what());
    return 3;
  }
  std::printf("cpp_api_check failures=%d\n", failures);
  return failures ? 1 : 0;
}
