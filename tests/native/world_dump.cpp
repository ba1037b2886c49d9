// Dumps the host build of csrc/mev_world.h + csrc/mev_routes.h (the exact code
// the gfx950 kernels and the route builder run) for comparison with the
// reference's own outputs in tests/golden/static_lanes{2,3}.npz.
//   world_dump <lanes> <out_prefix>   writes <prefix>.grid (750*750 u8: bit0 road, bit1 yellow, bit2 line),
//   <prefix>.paths (P*P*160*2 f32), <prefix>.intent (P*P i32), <prefix>.spawn (P*P*3 f32)
// and reads <prefix>.pts (n*2 f32) to write <prefix>.ptsout (n*2 u8: road, yellow).
#include <stdio.h>
#include <stdlib.h>

#include <string>
#include <vector>

#include "mev_routes.h"
#include "mev_world.h"

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    const int L = atoi(argv[1]);
    std::string pre = argv[2];
    const int irw = int(L * int(mev::LANE_WIDTH_PX));
    const int stop = irw + int(mev::CORNER_RADIUS);
    const float rw = L * mev::LANE_WIDTH_PX;
    std::vector<unsigned char> grid(750 * 750);
    for (int y = 0; y < 750; ++y)
        for (int x = 0; x < 750; ++x) {
            unsigned char v = 0;
            const bool r_int = mev::is_on_road_px(x, y, irw);
            const bool r_flt = mev::is_on_road(float(x), float(y), rw);
            if (r_int != r_flt) v |= 8;  // internal inconsistency flag
            if (r_int) v |= 1;
            if (mev::hits_yellow_line(float(x), float(y), rw)) v |= 2;
            if (mev::is_line_px(x, y, stop)) v |= 4;
            grid[y * 750 + x] = v;
        }
    FILE* f = fopen((pre + ".grid").c_str(), "wb");
    fwrite(grid.data(), 1, grid.size(), f);
    fclose(f);
    auto pts = mev::build_lane_points(L);
    const int P = 8 * L;
    std::vector<float> paths(size_t(P) * P * 320), spawn(size_t(P) * P * 3);
    std::vector<int> intent(size_t(P) * P);
    for (int s = 0; s < P; ++s)
        for (int e = 0; e < P; ++e) {
            const int r = s * P + e;
            intent[r] = mev::generate_route(pts, L, s, e, &paths[size_t(r) * 320]);
            spawn[3 * r] = pts[s].x;
            spawn[3 * r + 1] = pts[s].y;
            spawn[3 * r + 2] = mev::spawn_heading(&paths[size_t(r) * 320]);
        }
    f = fopen((pre + ".paths").c_str(), "wb");
    fwrite(paths.data(), 4, paths.size(), f);
    fclose(f);
    f = fopen((pre + ".intent").c_str(), "wb");
    fwrite(intent.data(), 4, intent.size(), f);
    fclose(f);
    f = fopen((pre + ".spawn").c_str(), "wb");
    fwrite(spawn.data(), 4, spawn.size(), f);
    fclose(f);
    f = fopen((pre + ".pts").c_str(), "rb");
    if (f) {
        std::vector<float> p;
        float buf[2];
        while (fread(buf, 4, 2, f) == 2) { p.push_back(buf[0]); p.push_back(buf[1]); }
        fclose(f);
        std::vector<unsigned char> o(p.size());
        for (size_t k = 0; k < p.size() / 2; ++k) {
            o[2 * k] = mev::is_on_road(p[2 * k], p[2 * k + 1], rw);
            o[2 * k + 1] = mev::hits_yellow_line(p[2 * k], p[2 * k + 1], rw);
        }
        f = fopen((pre + ".ptsout").c_str(), "wb");
        fwrite(o.data(), 1, o.size(), f);
        fclose(f);
    }
    return 0;
}
