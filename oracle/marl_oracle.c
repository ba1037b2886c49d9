/*
 * marl_oracle.c — TEST INFRASTRUCTURE: a plain-C CPU restatement of the
 * reference simulator's hot path (IntersectionEnv::step + get_observations),
 * one environment at a time, the straightforward sequential way the reference
 * does it (literal LiDAR march, serial collision loops, glibc libm).
 *
 * Used only by tests/ (as the checker for the device path on random states),
 * __graft_entry__.smoke() and bench.py's cpu_baseline fallback ("port").  It
 * is never the product path.  It is pinned against the golden vectors that the
 * REAL reference produced (tests/test_oracle.py replays every scenario and
 * requires bit-exact agreement).
 *
 * Build: gcc -O2 -ffp-contract=off -shared -fPIC marl_oracle.c -lm
 * (no -march: plain SSE like the reference build, no FMA contraction).
 *
 * Every function cites the reference file:line it restates.
 */
#define _POSIX_C_SOURCE 199309L
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* reference cpp/constants.h:4-20 */
#define W 750
#define H 750
#define SCALE_ 12.0f
#define FPS_ 60.0f
#define CAR_LENGTH 54.0f
#define CAR_WIDTH 24.0f
#define WHEELBASE CAR_LENGTH
#define LANE_WIDTH_PX 42.0f
#define CORNER_RADIUS 84.0f
#define MAX_ACC 15.0f
#define MAX_STEERING_ANGLE 0.6108652381980153f
#define PHYSICS_MAX_SPEED 8.0f
#define PI_F 3.14159265358979323846f
#define NEIGHBORS 5 /* cpp/IntersectionEnv.h:19 */
#define PATH_LEN 160      /* every lane-layout route (RouteGen.cpp:160-237) */
#define MAX_PATH_LEN 4096 /* orc_add_route's bound (the device's, mev_world.h MAX_PATH_LEN) */
#define MAXCARS 256

enum { ST_ALIVE = 0, ST_DEAD = 1, ST_SUCCESS = 2, ST_CRASH_WALL = 3, ST_CRASH_LINE = 4, ST_CRASH_CAR = 5 };

typedef struct {
    float x, y, v, h, acc, steer, sx, sy, sv, sh, prev_dist, pa0, pa1;
    int32_t path_index, route, intention, alive;
    float len, wid; /* Car::length / Car::width, cpp/Car.h:19-20 (default 54 x 24) */
} orc_car;

typedef struct {
    float x, y;
    char dir;
} lane_pt;

typedef struct orc_env {
    int lanes, n, rays, obs_dim, use_team, respawn, max_steps, traffic, max_npcs;
    float fov, maxd, step, density;
    float rc[8];
    int P;               /* 8 * lanes lane points */
    lane_pt* pts;
    float* paths;        /* the P*P lane-layout routes ([160][2] each), then orc_add_route's ([n][2] each) */
    size_t* poff;        /* [nroutes]: float offset of each route's path in paths */
    size_t pfloats;      /* floats used in paths */
    int* intent;         /* [nroutes] */
    int* plen;           /* [nroutes]: points of each path (Car.path.size(); 160 for the lane routes) */
    int nroutes;
    float* rel;          /* [rays] */
    uint8_t* line_grid;  /* [750*750] LineMask */
    int* troutes;        /* traffic route ids */
    int ntr;
    orc_car ego[MAXCARS];
    orc_car npc[MAXCARS];
    int nnpc;
    int step_count;
    float* lidar;        /* [n][rays] distances */
} orc_env;

/* ---------------------------------------------------------------- helpers */
/* wrap_angle_rad, cpp/IntersectionEnv.cpp:9-13 (== TrafficFlow.cpp:8-12) */
static float wrap_angle(float a) {
    a = fmodf(a + PI_F, 2.0f * PI_F);
    if (a < 0) a += 2.0f * PI_F;
    return a - PI_F;
}

/* ---------------------------------------------------- lane layout / routes */
/* build_lane_layout_cpp, cpp/RouteGen.cpp:7-53.  IN_k -> k-1, OUT_k -> 4L+k-1 */
static void build_points(orc_env* e) {
    const char dirs[4] = {'N', 'E', 'S', 'W'};
    const float CX = W * 0.5f, CY = H * 0.5f, M = 30.0f;
    e->P = 8 * e->lanes;
    e->pts = (lane_pt*)calloc((size_t)e->P, sizeof(lane_pt));
    for (int d = 0; d < 4; ++d)
        for (int j = 0; j < e->lanes; ++j) {
            float off = LANE_WIDTH_PX * (0.5f + (float)j);
            float ix, iy, ox, oy;
            char c = dirs[d];
            if (c == 'N') { ix = CX - off; iy = M; ox = CX + off; oy = M; }
            else if (c == 'S') { ix = CX + off; iy = H - M; ox = CX - off; oy = H - M; }
            else if (c == 'E') { ix = W - M; iy = CY - off; ox = W - M; oy = CY + off; }
            else { ix = M; iy = CY + off; ox = M; oy = CY - off; }
            int k = d * e->lanes + j;
            e->pts[k].x = ix; e->pts[k].y = iy; e->pts[k].dir = c;
            e->pts[4 * e->lanes + k].x = ox; e->pts[4 * e->lanes + k].y = oy; e->pts[4 * e->lanes + k].dir = c;
        }
}

static char opp(char d) { return d == 'N' ? 'S' : d == 'S' ? 'N' : d == 'E' ? 'W' : 'E'; }
static char lft(char d) { return d == 'N' ? 'E' : d == 'E' ? 'S' : d == 'S' ? 'W' : 'N'; }
static char rgt(char d) { return d == 'N' ? 'W' : d == 'W' ? 'S' : d == 'S' ? 'E' : 'N'; }

/* determine_intent, cpp/RouteGen.cpp:55-87 */
static int intent_of(char s, char t) {
    if (t == opp(s)) return 0;
    if (t == lft(s)) return 1;
    if (t == rgt(s)) return 2;
    return 1;
}

/* project_to_box, cpp/RouteGen.cpp:89-101 */
static void project_box(float x, float y, int lanes, float* ox, float* oy) {
    const float CX = W * 0.5f, CY = H * 0.5f;
    float tb = lanes * LANE_WIDTH_PX;
    float l = CX - tb, r = CX + tb, t = CY - tb, b = CY + tb;
    if (y < t) { *ox = x; *oy = t; return; }
    if (y > b) { *ox = x; *oy = b; return; }
    if (x < l) { *ox = l; *oy = y; return; }
    *ox = r; *oy = y;
}

/* generate_path_cpp, cpp/RouteGen.cpp:111-205 (bezier_point :103-109) */
static void gen_path(const orc_env* e, int s, int t, int intent, float* out) {
    const float CX = W * 0.5f, CY = H * 0.5f;
    const lane_pt* ps = &e->pts[s];
    const lane_pt* pe = &e->pts[t];
    float enx, eny, exx, exy;
    project_box(ps->x, ps->y, e->lanes, &enx, &eny);
    project_box(pe->x, pe->y, e->lanes, &exx, &exy);
    int o = 0;
#define PUSH(a, b) do { out[2 * o] = (a); out[2 * o + 1] = (b); ++o; } while (0)
    if (intent == 0 || intent == 1) {
        for (int i = 0; i < 50; ++i) {
            float tt = (float)i / 50.0f;
            PUSH(ps->x + (enx - ps->x) * tt, ps->y + (eny - ps->y) * tt);
        }
        for (int i = 0; i < 60; ++i) {
            float tt = (float)i / 60.0f;
            if (intent == 0) {
                PUSH(enx + (exx - enx) * tt, eny + (exy - eny) * tt);
            } else {
                float bx = (1 - tt) * (1 - tt) * enx + 2 * (1 - tt) * tt * CX + tt * tt * exx;
                float by = (1 - tt) * (1 - tt) * eny + 2 * (1 - tt) * tt * CY + tt * tt * exy;
                PUSH(bx, by);
            }
        }
        for (int i = 0; i < 50; ++i) {
            float tt = (float)i / 50.0f;
            PUSH(exx + (pe->x - exx) * tt, exy + (pe->y - exy) * tt);
        }
        return;
    }
    float rhw = e->lanes * LANE_WIDTH_PX;
    float ccx, ccy, th0, th1;
    if (ps->dir == 'N') { ccx = CX - rhw - CORNER_RADIUS; ccy = CY - rhw - CORNER_RADIUS; th0 = 0.0f; th1 = PI_F / 2.0f; }
    else if (ps->dir == 'E') { ccx = CX + rhw + CORNER_RADIUS; ccy = CY - rhw - CORNER_RADIUS; th0 = PI_F / 2.0f; th1 = PI_F; }
    else if (ps->dir == 'S') { ccx = CX + rhw + CORNER_RADIUS; ccy = CY + rhw + CORNER_RADIUS; th0 = PI_F; th1 = 3.0f * PI_F / 2.0f; }
    else { ccx = CX - rhw - CORNER_RADIUS; ccy = CY + rhw + CORNER_RADIUS; th0 = -PI_F / 2.0f; th1 = 0.0f; }
    float r = CORNER_RADIUS + 0.5f * LANE_WIDTH_PX;
    float asx = ccx + r * cosf(th0), asy = ccy + r * sinf(th0);
    float aex = ccx + r * cosf(th1), aey = ccy + r * sinf(th1);
    for (int i = 0; i < 50; ++i) {
        float tt = (float)i / 50.0f;
        PUSH(ps->x + (asx - ps->x) * tt, ps->y + (asy - ps->y) * tt);
    }
    for (int i = 0; i < 60; ++i) {
        float tt = (float)i / 60.0f;
        float th = th0 + (th1 - th0) * tt;
        PUSH(ccx + r * cosf(th), ccy + r * sinf(th));
    }
    for (int i = 0; i < 50; ++i) {
        float tt = (float)i / 50.0f;
        PUSH(aex + (pe->x - aex) * tt, aey + (pe->y - aey) * tt);
    }
#undef PUSH
}

/* LineMask::generate / draw_thick_line, cpp/LineMask.cpp:14-72 */
static void set_px(uint8_t* g, int x, int y) {
    if (x < 0 || x >= W || y < 0 || y >= H) return;
    g[y * W + x] = 1;
}
static void thick_line(uint8_t* g, int x0, int y0, int x1, int y1) {
    const int half = 1; /* thickness 2 */
    if (x0 == x1) {
        int ya = y0 < y1 ? y0 : y1, yb = y0 < y1 ? y1 : y0;
        for (int y = ya; y <= yb; ++y)
            for (int d = -half; d <= half; ++d) set_px(g, x0 + d, y);
    } else if (y0 == y1) {
        int xa = x0 < x1 ? x0 : x1, xb = x0 < x1 ? x1 : x0;
        for (int x = xa; x <= xb; ++x)
            for (int d = -half; d <= half; ++d) set_px(g, x, y0 + d);
    }
}
static void build_line_grid(orc_env* e) {
    e->line_grid = (uint8_t*)calloc((size_t)W * H, 1);
    int cx = W / 2, cy = H / 2, rw = (int)(e->lanes * (int)LANE_WIDTH_PX), cr = (int)CORNER_RADIUS;
    int so = rw + cr;
    uint8_t* g = e->line_grid;
    thick_line(g, cx - 2, 0, cx - 2, cy - so);
    thick_line(g, cx + 2, 0, cx + 2, cy - so);
    thick_line(g, cx - 2, H, cx - 2, cy + so);
    thick_line(g, cx + 2, H, cx + 2, cy + so);
    thick_line(g, 0, cy - 2, cx - so, cy - 2);
    thick_line(g, 0, cy + 2, cx - so, cy + 2);
    thick_line(g, W, cy - 2, cx + so, cy - 2);
    thick_line(g, W, cy + 2, cx + so, cy + 2);
}
static int is_line(const orc_env* e, int x, int y) { /* LineMask.h:15-18 */
    if (x < 0 || x >= W || y < 0 || y >= H) return 0;
    return e->line_grid[y * W + x] != 0;
}

/* RoadGeometry::is_on_road, cpp/RoadGeometry.h:19-58 */
static int on_road(const orc_env* e, float x, float y) {
    const float CX = W * 0.5f, CY = H * 0.5f;
    const float rw = e->lanes * LANE_WIDTH_PX, cr = CORNER_RADIUS, r2 = cr * cr;
    const float gx[4] = {CX - rw - cr, CX + rw + cr, CX - rw - cr, CX + rw + cr};
    const float gy[4] = {CY - rw - cr, CY - rw - cr, CY + rw + cr, CY + rw + cr};
    for (int k = 0; k < 4; ++k) {
        float dx = x - gx[k], dy = y - gy[k];
        if (dx * dx + dy * dy <= r2) return 0;
    }
    if ((x >= CX - rw && x <= CX + rw) || (y >= CY - rw && y <= CY + rw)) return 1;
    if (x >= CX - rw - cr && x <= CX - rw && y >= CY - rw - cr && y <= CY - rw) return 1;
    if (x >= CX + rw && x <= CX + rw + cr && y >= CY - rw - cr && y <= CY - rw) return 1;
    if (x >= CX - rw - cr && x <= CX - rw && y >= CY + rw && y <= CY + rw + cr) return 1;
    if (x >= CX + rw && x <= CX + rw + cr && y >= CY + rw && y <= CY + rw + cr) return 1;
    return 0;
}

/* RoadGeometry::hits_yellow_line, cpp/RoadGeometry.h:60-67 */
static int yellow(const orc_env* e, float x, float y) {
    float cx = W * 0.5f, cy = H * 0.5f, gap = 2.0f, rw = e->lanes * LANE_WIDTH_PX;
    if (fabsf(x - cx) <= gap && fabsf(y - cy) > rw) return 1;
    if (fabsf(y - cy) <= gap && fabsf(x - cx) > rw) return 1;
    return 0;
}

/* ------------------------------------------------------------------ cars */
static const float* path_of(const orc_env* e, const orc_car* c) { return e->paths + e->poff[c->route]; }
static int len_of(const orc_env* e, const orc_car* c) { return e->plen[c->route]; } /* path.size() */

/* Car::update, cpp/Car.cpp:9-40 */
static void car_update(orc_car* c, float thr, float st, float dt) {
    c->acc = thr * MAX_ACC;
    float target = st * MAX_STEERING_ANGLE;
    c->steer += (target - c->steer) * 0.2f;
    if (thr == 0.0f) c->v *= 0.95f;
    c->v += c->acc * dt;
    if (c->v < 0.0f) c->v = 0.0f;
    if (c->v > PHYSICS_MAX_SPEED) c->v = PHYSICS_MAX_SPEED;
    if (fabsf(c->v) > 0.1f) {
        float ang_vel = (c->v / WHEELBASE) * tanf(c->steer);
        c->h += ang_vel;
    }
    c->h = fmodf(c->h + PI_F, 2.0f * PI_F);
    if (c->h < 0) c->h += 2.0f * PI_F;
    c->h -= PI_F;
    c->x += c->v * cosf(c->h);
    c->y -= c->v * sinf(c->h);
}

/* Car::update_path_index, cpp/Car.cpp:47-74 */
static void update_path_index(const orc_env* e, orc_car* c) {
    const float* p = path_of(e, c);
    int s = c->path_index < 0 ? 0 : c->path_index;
    const int L = len_of(e, c);
    int end = s + 50 < L ? s + 50 : L;
    float best = INFINITY;
    int bi = s;
    for (int i = s; i < end; ++i) {
        float dx = p[2 * i] - c->x, dy = p[2 * i + 1] - c->y;
        float d = dx * dx + dy * dy;
        if (d < best) { best = d; bi = i; }
    }
    c->path_index = bi;
}

/* Car::respawn, cpp/Car.cpp:76-84 */
static void respawn(orc_car* c) {
    c->x = c->sx; c->y = c->sy; c->v = c->sv; c->h = c->sh;
    c->alive = 1; c->path_index = 0; c->prev_dist = 0.0f; c->pa0 = 0.0f; c->pa1 = 0.0f;
    c->acc = 0.0f; c->steer = 0.0f;
}

/* Car::corners, cpp/Car.cpp:86-103 (the car's own width / length) */
static void corners(const orc_car* c, float* px, float* py) {
    const float hx = c->wid * 0.5f, hy = c->len * 0.5f;
    const float ca = cosf(c->h), sa = sinf(c->h);
    const float lx[4] = {hy, hy, -hy, -hy}, ly[4] = {hx, -hx, -hx, hx};
    for (int k = 0; k < 4; ++k) {
        px[k] = c->x + lx[k] * ca - ly[k] * sa;
        py[k] = c->y + lx[k] * sa + ly[k] * ca;
    }
}

/* project + Car::check_collision, cpp/Car.cpp:105-141 */
static void project(const float* px, const float* py, float ax, float ay, float* mn, float* mx) {
    float a = INFINITY, b = -INFINITY;
    for (int k = 0; k < 4; ++k) {
        float p = px[k] * ax + py[k] * ay;
        a = (p < a) ? p : a;
        b = (b < p) ? p : b;
    }
    *mn = a; *mx = b;
}
static int collide(const orc_car* a, const orc_car* b) {
    float ax[4], ay[4], bx[4], by[4];
    corners(a, ax, ay);
    corners(b, bx, by);
    float c1 = cosf(a->h), s1 = sinf(a->h), c2 = cosf(b->h), s2 = sinf(b->h);
    float axs[4][2] = {{c1, s1}, {-s1, c1}, {c2, s2}, {-s2, c2}};
    for (int k = 0; k < 4; ++k) {
        float m1, M1, m2, M2;
        project(ax, ay, axs[k][0], axs[k][1], &m1, &M1);
        project(bx, by, axs[k][0], axs[k][1], &m2, &M2);
        if (M1 < m2 || M2 < m1) return 0;
    }
    return 1;
}

/* ----------------------------------------------------------------- LiDAR */
/* Lidar::update, cpp/Lidar.cpp:16-90 — the literal sequential march */
static void lidar_update(const orc_env* e, const orc_car* self, int self_idx, const orc_car* obs, int nobs, float* out) {
    const float cx = self->x, cy = self->y, hd = self->h;
    for (int i = 0; i < e->rays; ++i) {
        float ang = hd + e->rel[i];
        float dx = cosf(ang), dy = -sinf(ang);
        int hit = 0;
        float fd = e->maxd;
        for (float dist = 0.0f; dist < e->maxd; dist += e->step) {
            int px = (int)(cx + dx * dist), py = (int)(cy + dy * dist);
            if (px < 0 || px >= W || py < 0 || py >= H) break;
            if (dist > 0.0f && !on_road(e, (float)px, (float)py)) { hit = 1; fd = dist; break; }
            if (dist > 0.0f) {
                int col = 0;
                for (int j = 0; j < nobs; ++j) {
                    const orc_car* c = &obs[j];
                    if (j == self_idx) continue;
                    if (fabsf(c->x - cx) < 1e-3f && fabsf(c->y - cy) < 1e-3f && fabsf(c->h - hd) < 1e-3f) continue;
                    float ca = cosf(c->h), sa = sinf(c->h);
                    float hl = c->len * 0.5f, hw = c->wid * 0.5f; /* Lidar.cpp:67-68 */
                    float ex = fabsf(ca) * hl + fabsf(sa) * hw;
                    float ey = fabsf(sa) * hl + fabsf(ca) * hw;
                    if ((float)px >= c->x - ex && (float)px <= c->x + ex && (float)py >= c->y - ey && (float)py <= c->y + ey) {
                        col = 1;
                        break;
                    }
                }
                if (col) { hit = 1; fd = dist; break; }
            }
        }
        out[i] = hit ? fd : e->maxd;
    }
}

/* ---------------------------------------------------------- NPC traffic */
/* get_front_car_dist_tf, cpp/TrafficFlow.cpp:22-47 */
static float front_dist(const orc_env* e, int k) {
    const orc_car* s = &e->npc[k];
    float md = 1e9f, vx = cosf(s->h), vy = -sinf(s->h);
    for (int j = 0; j < e->nnpc; ++j) {
        const orc_car* o = &e->npc[j];
        if (j == k || !o->alive) continue;
        float dx = o->x - s->x, dy = o->y - s->y;
        float dist = hypotf(dx, dy);
        if (dist > 80.0f) continue;
        float dot = (dx * vx + dy * vy) / (dist + 1e-5f);
        if (dot > 0.8f) {
            float ad = fabsf(wrap_angle(s->h - o->h));
            if (ad < (45.0f * PI_F / 180.0f))
                if (dist < md) md = dist;
        }
    }
    return md;
}

/* plan_npc_action_tf, cpp/TrafficFlow.cpp:49-196 */
static void plan_npc(const orc_env* e, int k, float* thr_out, float* st_out) {
    const orc_car* n = &e->npc[k];
    const float* path = path_of(e, n);
    float steer = 0.0f;
    {
        int ti = n->path_index + 12;
        if (ti > len_of(e, n) - 1) ti = len_of(e, n) - 1;
        float dx = path[2 * ti] - n->x, dy = path[2 * ti + 1] - n->y;
        float err = wrap_angle(atan2f(-dy, dx) - n->h);
        float v = err * 3.0f;
        v = (1.0f < v) ? 1.0f : v;
        steer = (v < -1.0f) ? -1.0f : v;
    }
    const float target = PHYSICS_MAX_SPEED * 0.4f;
    float acc = 0.0f;
    if (n->v < target) acc = 0.5f;
    else if (n->v > target + 1.0f) acc = -0.1f;
    float fd = front_dist(e, k);
    if (fd < 30.0f) acc = -1.0f;
    else if (fd < 50.0f) acc = (-0.2f < acc) ? -0.2f : acc;

    int conflict = 0;
    float minc = 1e9f;
    const float SAFE = CAR_WIDTH * 2.0f, SAFE_SQ = SAFE * SAFE;
    float mdc = hypotf(n->x - W * 0.5f, n->y - H * 0.5f);
    int s = n->path_index, end = s + 120 < len_of(e, n) ? s + 120 : len_of(e, n);
    for (int i = s; i < end; ++i) {
        float gx = path[2 * i], gy = path[2 * i + 1];
        for (int j = 0; j < e->nnpc; ++j) {
            const orc_car* o = &e->npc[j];
            if (j == k || !o->alive) continue;
            float dxo = o->x - gx, dyo = o->y - gy;
            if (dxo * dxo + dyo * dyo < SAFE_SQ) {
                float ad = fabsf(wrap_angle(n->h - o->h));
                if (ad < (60.0f * PI_F / 180.0f)) continue;
                {
                    float dxt = o->x - n->x, dyt = o->y - n->y;
                    float dto = hypotf(dxt, dyt);
                    if (dto > 1e-5f) {
                        float mdx = cosf(n->h), mdy = -sinf(n->h);
                        float tpm = 2.0f * PI_F - ad;
                        float adn = (tpm < ad) ? tpm : ad;
                        int par = (adn < (30.0f * PI_F / 180.0f)) || (adn > (150.0f * PI_F / 180.0f));
                        if (par) {
                            float lon = dxt * mdx + dyt * mdy;
                            float lsq = dto * dto - lon * lon;
                            lsq = (0.0f < lsq) ? lsq : 0.0f;
                            float lat = sqrtf(lsq);
                            int side = fabsf(lat) < (LANE_WIDTH_PX * 1.5f);
                            int near = fabsf(lon) < (CAR_LENGTH * 2.0f);
                            if (side && near) {
                                float fdist = 20.0f;
                                float mfx = n->x + mdx * fdist, mfy = n->y + mdy * fdist;
                                float odx = cosf(o->h), ody = -sinf(o->h);
                                float ofx = o->x + odx * fdist, ofy = o->y + ody * fdist;
                                float fdx = ofx - mfx, fdy = ofy - mfy;
                                float fm = hypotf(fdx, fdy);
                                if (fm > 1e-5f) {
                                    float fl = fdx * mdx + fdy * mdy;
                                    float flsq = fm * fm - fl * fl;
                                    flsq = (0.0f < flsq) ? flsq : 0.0f;
                                    float flat = sqrtf(flsq);
                                    if (fabsf(flat - lat) < (LANE_WIDTH_PX * 0.5f)) continue;
                                }
                            }
                        }
                    }
                }
                int yield = 0;
                float odc = hypotf(o->x - W * 0.5f, o->y - H * 0.5f);
                float dtc = hypotf(gx - n->x, gy - n->y);
                if (dtc < 15.0f) yield = 1;
                else if (n->v < 1.0f && o->v > 3.0f && odc < mdc + 25.0f) yield = 1;
                else if (odc < mdc - 5.0f) yield = 1;
                else if (fabsf(odc - mdc) <= 5.0f) { if (k < j) yield = 1; } /* address order */
                if (yield) {
                    conflict = 1;
                    if (dtc < minc) minc = dtc;
                }
            }
        }
        if (conflict) break;
    }
    float thr = acc;
    if (conflict) {
        if (minc < 35.0f) thr = -1.0f;
        else if (minc < 60.0f) thr = -0.8f;
        else thr = (0.0f < thr) ? 0.0f : thr;
    }
    *thr_out = thr;
    *st_out = steer;
}

/* try_spawn_traffic_car, cpp/TrafficFlow.cpp:240-315 (route decided by the caller) */
static void spawn_npc(orc_env* e, int troute) {
    if (troute < 0 || troute >= e->ntr) return;
    int rid = e->troutes[troute];
    const float* p = e->paths + e->poff[rid];
    /* the route's start lane point; a route of the caller's own (orc_add_route) starts at its first point */
    float sx = rid < e->P * e->P ? e->pts[rid / e->P].x : p[0], sy = rid < e->P * e->P ? e->pts[rid / e->P].y : p[1];
    const float md = CAR_LENGTH * 2.5f, md2 = md * md;
    for (int i = 0; i < e->n; ++i) {
        float dx = e->ego[i].x - sx, dy = e->ego[i].y - sy;
        if (dx * dx + dy * dy < md2) return;
    }
    for (int i = 0; i < e->nnpc; ++i) {
        float dx = e->npc[i].x - sx, dy = e->npc[i].y - sy;
        if (dx * dx + dy * dy < md2) return;
    }
    if (e->nnpc >= e->max_npcs) return;
    orc_car c;
    memset(&c, 0, sizeof(c));
    c.x = sx; c.y = sy; c.v = 0.0f;
    c.h = atan2f(-(p[3] - p[1]), p[2] - p[0]);
    c.sx = c.x; c.sy = c.y; c.sv = 0.0f; c.sh = c.h;
    c.alive = 1; c.intention = e->intent[rid]; c.route = rid; c.path_index = 0;
    c.len = CAR_LENGTH; c.wid = CAR_WIDTH; /* a new Car, cpp/Car.h:19-20 */
    e->npc[e->nnpc++] = c;
}

/* update_traffic_flow, cpp/TrafficFlow.cpp:317-367 */
static void traffic_flow(orc_env* e, float dt, int spawn_route) {
    spawn_npc(e, spawn_route);
    for (int k = 0; k < e->nnpc; ++k) {
        orc_car* n = &e->npc[k];
        if (!n->alive) continue;
        update_path_index(e, n);
        float thr, st;
        plan_npc(e, k, &thr, &st);
        car_update(n, thr, st, dt);
        update_path_index(e, n);
    }
    for (int i = 0; i < e->nnpc; ++i) {
        if (!e->npc[i].alive) continue;
        for (int j = i + 1; j < e->nnpc; ++j) {
            if (!e->npc[j].alive) continue;
            if (collide(&e->npc[i], &e->npc[j])) { e->npc[i].alive = 0; e->npc[j].alive = 0; }
        }
    }
    int w = 0;
    for (int i = 0; i < e->nnpc; ++i) {
        orc_car* c = &e->npc[i];
        const float* p = path_of(e, c);
        const int L = len_of(e, c); /* path.back(), TrafficFlow.cpp:262-270 */
        int arrived = hypotf(c->x - p[2 * (L - 1)], c->y - p[2 * (L - 1) + 1]) < 20.0f;
        int oos = c->x < -100.0f || c->x > (float)W + 100.0f || c->y < -100.0f || c->y > (float)H + 100.0f;
        if (!c->alive || arrived || oos) continue;
        e->npc[w++] = *c;
    }
    e->nnpc = w;
}

/* ------------------------------------------------ std::sort (libstdc++) */
/* The neighbour sort of get_observations (cpp/IntersectionEnv.cpp:466-490) is
 * std::sort with `a.dist < b.dist`: NOT stable.  Restated from this image's
 * GCC 11 libstdc++ (bits/stl_algo.h __sort / __introsort_loop /
 * __unguarded_partition_pivot / __move_median_to_first / __unguarded_partition /
 * __final_insertion_sort, bits/stl_heap.h __make_heap / __adjust_heap /
 * __push_heap / __pop_heap / __sort_heap), which the reference build links: for
 * more than 16 neighbours with equal distances the order of equal neighbours is
 * the one these partitions leave, not the push order. */
typedef struct {
    float d;
    const orc_car* c;
} orc_nref; /* NeighborRef, IntersectionEnv.cpp:461-464 */

static void nr_swap(orc_nref* a, orc_nref* b) { orc_nref t = *a; *a = *b; *b = t; }

static void nr_push_heap(orc_nref* f, long hole, long top, orc_nref v) {
    long parent = (hole - 1) / 2;
    while (hole > top && f[parent].d < v.d) {
        f[hole] = f[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    f[hole] = v;
}

static void nr_adjust_heap(orc_nref* f, long hole, long len, orc_nref v) {
    const long top = hole;
    long sc = hole;
    while (sc < (len - 1) / 2) {
        sc = 2 * (sc + 1);
        if (f[sc].d < f[sc - 1].d) sc--;
        f[hole] = f[sc];
        hole = sc;
    }
    if ((len & 1) == 0 && sc == (len - 2) / 2) {
        sc = 2 * (sc + 1);
        f[hole] = f[sc - 1];
        hole = sc - 1;
    }
    nr_push_heap(f, hole, top, v);
}

/* __partial_sort(first, last, last): __heap_select (= __make_heap, its loop is empty) + __sort_heap */
static void nr_heapsort(orc_nref* f, long len) {
    if (len >= 2)
        for (long parent = (len - 2) / 2;; --parent) {
            nr_adjust_heap(f, parent, len, f[parent]);
            if (parent == 0) break;
        }
    for (long l = len; l > 1;) {
        --l;
        orc_nref v = f[l];
        f[l] = f[0];
        nr_adjust_heap(f, 0, l, v);
    }
}

static void nr_introsort_loop(orc_nref* first, orc_nref* last, int depth) {
    while (last - first > 16) {
        if (depth == 0) {
            nr_heapsort(first, last - first);
            return;
        }
        --depth;
        /* __unguarded_partition_pivot: median of (first+1, mid, last-1) into *first */
        orc_nref *a = first + 1, *b = first + (last - first) / 2, *c = last - 1;
        if (a->d < b->d) {
            if (b->d < c->d) nr_swap(first, b);
            else if (a->d < c->d) nr_swap(first, c);
            else nr_swap(first, a);
        } else if (a->d < c->d) nr_swap(first, a);
        else if (b->d < c->d) nr_swap(first, c);
        else nr_swap(first, b);
        /* __unguarded_partition(first + 1, last, first) */
        orc_nref *lo = first + 1, *hi = last;
        for (;;) {
            while (lo->d < first->d) ++lo;
            --hi;
            while (first->d < hi->d) --hi;
            if (!(lo < hi)) break;
            nr_swap(lo, hi);
            ++lo;
        }
        nr_introsort_loop(lo, last, depth);
        last = lo;
    }
}

static void nr_linear_insert(orc_nref* last) { /* __unguarded_linear_insert */
    orc_nref v = *last;
    orc_nref* next = last - 1;
    while (v.d < next->d) {
        *last = *next;
        last = next;
        --next;
    }
    *last = v;
}

static void nr_insertion_sort(orc_nref* first, orc_nref* last) { /* __insertion_sort */
    if (first == last) return;
    for (orc_nref* i = first + 1; i != last; ++i) {
        if (i->d < first->d) {
            orc_nref v = *i;
            memmove(first + 1, first, (size_t)(i - first) * sizeof(orc_nref));
            *first = v;
        } else {
            nr_linear_insert(i);
        }
    }
}

static void nr_std_sort(orc_nref* f, int n) {
    if (n <= 0) return;
    int lg = 0; /* std::__lg */
    while ((2 << lg) <= n) ++lg;
    nr_introsort_loop(f, f + n, 2 * lg);
    if (n > 16) { /* __final_insertion_sort */
        nr_insertion_sort(f, f + 16);
        for (orc_nref* i = f + 16; i != f + n; ++i) nr_linear_insert(i);
    } else {
        nr_insertion_sort(f, f + n);
    }
}

/* test hook: the permutation std::sort leaves on n distances (ids in push order) */
void orc_std_sort_perm(const float* d, int n, int* perm) {
    orc_nref* a = (orc_nref*)malloc(sizeof(orc_nref) * (size_t)(n > 0 ? n : 1));
    for (int k = 0; k < n; ++k) { a[k].d = d[k]; a[k].c = (const orc_car*)(uintptr_t)(k + 1); }
    nr_std_sort(a, n);
    for (int k = 0; k < n; ++k) perm[k] = (int)(uintptr_t)a[k].c - 1;
    free(a);
}

/* ---------------------------------------------------------- observation */
/* get_observations, cpp/IntersectionEnv.cpp:418-520 */
static void observe(const orc_env* e, float* obs) {
    const int D = e->obs_dim;
    memset(obs, 0, sizeof(float) * (size_t)e->n * (size_t)D);
    for (int i = 0; i < e->n; ++i) {
        const orc_car* c = &e->ego[i];
        float* row = obs + (size_t)i * D;
        if (!c->alive) continue;
        row[0] = c->x / (float)W;
        row[1] = c->y / (float)H;
        row[2] = c->v / PHYSICS_MAX_SPEED;
        row[3] = c->h / PI_F;
        const float* p = path_of(e, c);
        int ti = c->path_index + 10;
        if (ti > len_of(e, c) - 1) ti = len_of(e, c) - 1;
        float dx = p[2 * ti] - c->x, dy = p[2 * ti + 1] - c->y;
        row[4] = sqrtf(dx * dx + dy * dy) / (float)W;
        row[5] = wrap_angle(atan2f(-dy, dx) - c->h) / PI_F;
        /* neighbours: other alive egos, then alive NPCs (:466-488), std::sort by distance (:490) */
        orc_nref neigh[2 * MAXCARS];
        int cnt = 0;
        for (int j = 0; j < e->n; ++j) {
            if (j == i || !e->ego[j].alive) continue;
            float ddx = e->ego[j].x - c->x, ddy = e->ego[j].y - c->y;
            neigh[cnt].d = sqrtf(ddx * ddx + ddy * ddy);
            neigh[cnt++].c = &e->ego[j];
        }
        if (e->traffic)
            for (int j = 0; j < e->nnpc; ++j) {
                if (!e->npc[j].alive) continue;
                float ddx = e->npc[j].x - c->x, ddy = e->npc[j].y - c->y;
                neigh[cnt].d = sqrtf(ddx * ddx + ddy * ddy);
                neigh[cnt++].c = &e->npc[j];
            }
        nr_std_sort(neigh, cnt);
        int take = cnt < NEIGHBORS ? cnt : NEIGHBORS;
        for (int k = 0; k < take; ++k) {
            const orc_car* o = neigh[k].c;
            float* f = row + 6 + 5 * k;
            f[0] = (o->x - c->x) / (float)W;
            f[1] = (o->y - c->y) / (float)H;
            f[2] = (o->v - c->v) / PHYSICS_MAX_SPEED;
            f[3] = wrap_angle(o->h - c->h) / PI_F;
            f[4] = (float)o->intention;
        }
        const float inv = (e->maxd > 0.0f) ? (1.0f / e->maxd) : 0.0f;
        for (int b = 0; b < e->rays && 31 + b < D; ++b) row[31 + b] = e->lidar[i * e->rays + b] * inv;
    }
}

/* ------------------------------------------------------------ public API */
orc_env* orc_create(int lanes, int n, int rays, float fov, float maxd, float step, int obs_dim, int use_team,
                    int respawn_on, int max_steps, int traffic, float density, const float* rc, int max_npcs) {
    if (n < 0 || n > MAXCARS || rays < 1 || max_npcs < 0 || max_npcs > MAXCARS) return NULL;  /* n = 0: an env without egos */
    orc_env* e = (orc_env*)calloc(1, sizeof(orc_env));
    e->lanes = lanes; e->n = n; e->rays = rays; e->fov = fov; e->maxd = maxd; e->step = step;
    e->obs_dim = obs_dim > 0 ? obs_dim : 31 + rays;
    e->use_team = use_team; e->respawn = respawn_on; e->max_steps = max_steps;
    e->traffic = traffic; e->density = density < 0.0f ? 0.0f : density; e->max_npcs = max_npcs;
    memcpy(e->rc, rc, sizeof(e->rc));
    build_points(e);
    e->nroutes = e->P * e->P;
    e->paths = (float*)calloc((size_t)e->P * e->P * 2 * PATH_LEN, sizeof(float));
    e->intent = (int*)calloc((size_t)e->P * e->P, sizeof(int));
    e->plen = (int*)calloc((size_t)e->P * e->P, sizeof(int));
    e->poff = (size_t*)calloc((size_t)e->P * e->P, sizeof(size_t));
    for (int r = 0; r < e->P * e->P; ++r) { e->plen[r] = PATH_LEN; e->poff[r] = (size_t)r * 2 * PATH_LEN; }
    e->pfloats = (size_t)e->P * e->P * 2 * PATH_LEN;
    for (int s = 0; s < e->P; ++s)
        for (int t = 0; t < e->P; ++t) {
            int r = s * e->P + t;
            e->intent[r] = intent_of(e->pts[s].dir, e->pts[t].dir);
            gen_path(e, s, t, e->intent[r], e->paths + (size_t)r * 2 * PATH_LEN);
        }
    /* LiDAR beam offsets, cpp/IntersectionEnv.cpp:119-127 */
    e->rel = (float*)calloc((size_t)rays, sizeof(float));
    {
        float sa = -fov * 0.5f;
        float sd = (rays > 1) ? (fov / (float)(rays - 1)) : 0.0f;
        for (int i = 0; i < rays; ++i) {
            float deg = sa + i * sd;
            e->rel[i] = deg * PI_F / 180.0f;
        }
    }
    build_line_grid(e);
    e->troutes = (int*)calloc((size_t)e->P * e->P, sizeof(int));
    e->lidar = (float*)calloc((size_t)n * rays, sizeof(float));
    return e;
}

void orc_destroy(orc_env* e) {
    if (!e) return;
    free(e->pts); free(e->paths); free(e->intent); free(e->plen); free(e->poff); free(e->rel); free(e->line_grid); free(e->troutes); free(e->lidar);
    free(e);
}

int orc_route_id(const orc_env* e, int s, int t) { return s * e->P + t; }
int orc_num_points(const orc_env* e) { return e->P; }
int orc_route_len(const orc_env* e, int r) { return e->plen[r]; }

void orc_route_path(const orc_env* e, int r, float* out, int* intent) {
    memcpy(out, e->paths + e->poff[r], sizeof(float) * 2 * (size_t)e->plen[r]);
    *intent = e->intent[r];
}

/* A route of the caller's own (the reference's Car.path is a plain read-write
 * vector, cpp/Car.h:26, cpp/bindings.cpp:29; every function above reads a car's
 * path through path_of, bounded by its size, len_of): n points (2 <= n <= MAX_PATH_LEN)
 * appended to the table, returns its id. */
int orc_add_route(orc_env* e, const float* path, int n, int intent) {
    if (n < 2 || n > MAX_PATH_LEN) return -1;
    float* np = (float*)realloc(e->paths, (e->pfloats + 2 * (size_t)n) * sizeof(float));
    if (!np) return -1;
    e->paths = np;
    size_t* no = (size_t*)realloc(e->poff, (size_t)(e->nroutes + 1) * sizeof(size_t));
    if (!no) return -1;
    e->poff = no;
    int* ni = (int*)realloc(e->intent, (size_t)(e->nroutes + 1) * sizeof(int));
    if (!ni) return -1;
    e->intent = ni;
    int* nl = (int*)realloc(e->plen, (size_t)(e->nroutes + 1) * sizeof(int));
    if (!nl) return -1;
    e->plen = nl;
    e->poff[e->nroutes] = e->pfloats;
    memcpy(e->paths + e->pfloats, path, sizeof(float) * 2 * (size_t)n);
    e->pfloats += 2 * (size_t)n;
    e->intent[e->nroutes] = intent;
    e->plen[e->nroutes] = n;
    return e->nroutes++;
}

/* Lidar::rel_angles written by the caller (read-write, cpp/bindings.cpp:91): the
 * first `rays` offsets are the beams' (Lidar.cpp:25). */
void orc_set_rel_angles(orc_env* e, const float* rel) { memcpy(e->rel, rel, sizeof(float) * (size_t)e->rays); }

void orc_set_traffic_routes(orc_env* e, const int* ids, int m) {
    e->ntr = m;
    memcpy(e->troutes, ids, sizeof(int) * (size_t)m);
}

/* IntersectionEnv::reset + add_car_with_route, cpp/IntersectionEnv.cpp:66-131 */
void orc_reset(orc_env* e, const int* routes) {
    for (int i = 0; i < e->n; ++i) {
        orc_car* c = &e->ego[i];
        memset(c, 0, sizeof(*c));
        int r = routes[i];
        const float* p = e->paths + e->poff[r];
        c->route = r;
        c->x = e->pts[r / e->P].x; c->y = e->pts[r / e->P].y; c->v = 0.0f;
        c->h = atan2f(-(p[3] - p[1]), p[2] - p[0]);
        c->sx = c->x; c->sy = c->y; c->sv = 0.0f; c->sh = c->h;
        c->alive = 1; c->intention = e->intent[r];
        c->len = CAR_LENGTH; c->wid = CAR_WIDTH; /* a new Car, cpp/Car.h:19-20 */
        for (int b = 0; b < e->rays; ++b) e->lidar[i * e->rays + b] = e->maxd;
    }
    e->nnpc = 0;
    e->step_count = 0;
}

void orc_set_state(orc_env* e, const orc_car* egos, const orc_car* npcs, int nnpc, int step_count) {
    memcpy(e->ego, egos, sizeof(orc_car) * (size_t)e->n);
    memcpy(e->npc, npcs, sizeof(orc_car) * (size_t)nnpc);
    e->nnpc = nnpc;
    e->step_count = step_count;
    for (int b = 0; b < e->n * e->rays; ++b) e->lidar[b] = e->maxd;
}

void orc_get_state(const orc_env* e, orc_car* egos, orc_car* npcs, int* nnpc, int* step_count) {
    memcpy(egos, e->ego, sizeof(orc_car) * (size_t)e->n);
    memcpy(npcs, e->npc, sizeof(orc_car) * (size_t)e->nnpc);
    *nnpc = e->nnpc;
    *step_count = e->step_count;
}

void orc_observe(const orc_env* e, float* obs) { observe(e, obs); }

/* IntersectionEnv::step, cpp/IntersectionEnv.cpp:133-392.  flags: term, trunc, alive, step */
void orc_step(orc_env* e, const float* actions, float dt, int spawn_route, float* obs, float* rew, uint8_t* done,
              uint8_t* status, int32_t* flags) {
    const int n = e->n;
    const float max_progress = hypotf((float)W, (float)H);
    int step_no = ++e->step_count;
    if (e->traffic) traffic_flow(e, dt, spawn_route);
    for (int i = 0; i < n; ++i) { rew[i] = 0.0f; done[i] = 0; status[i] = ST_ALIVE; }
    for (int i = 0; i < n; ++i) {
        orc_car* c = &e->ego[i];
        if (!c->alive) continue;
        car_update(c, actions[2 * i], actions[2 * i + 1], dt);
        update_path_index(e, c);
        /* compute_progress / compute_stuck / compute_smooth, :15-46 */
        const float* p = path_of(e, c);
        const int L = len_of(e, c); /* goal = path.back(), :16-17 */
        float cur = hypotf(c->x - p[2 * (L - 1)], c->y - p[2 * (L - 1) + 1]);
        float rp = 0.0f;
        if (c->prev_dist > 0.0f) {
            float prog = c->prev_dist - cur;
            float nrm = (max_progress > 0.0f) ? (prog / max_progress) : 0.0f;
            rp = e->rc[0] * nrm;
        }
        c->prev_dist = cur;
        float sms = (c->v * FPS_) / SCALE_;
        float rs = (sms < e->rc[1]) ? e->rc[2] : 0.0f;
        float an = c->acc / MAX_ACC, sn = c->steer / MAX_STEERING_ANGLE;
        float d0 = an - c->pa0, d1 = sn - c->pa1;
        float rsm = e->rc[6] * (d0 * d0 + d1 * d1);
        c->pa0 = an; c->pa1 = sn;
        rew[i] = rp + rs + rsm;
    }
    for (int i = 0; i < n; ++i) { /* status, :165-290 */
        orc_car* c = &e->ego[i];
        if (!c->alive) { done[i] = 1; status[i] = ST_DEAD; continue; }
        const float* p = path_of(e, c);
        const int L = len_of(e, c); /* path[size - 1], path[size - 2], :177-182 */
        float ex = p[2 * (L - 1)], ey = p[2 * (L - 1) + 1];
        float dxr = ex - p[2 * (L - 2)], dyr = ey - p[2 * (L - 2) + 1];
        int succ;
        if (fabsf(dxr) > fabsf(dyr)) succ = fabsf(c->y - ey) < 15.0f && fabsf(c->x - ex) < 40.0f;
        else succ = fabsf(c->x - ex) < 15.0f && fabsf(c->y - ey) < 40.0f;
        if (succ) { done[i] = 1; status[i] = ST_SUCCESS; continue; }
        float px[4], py[4];
        corners(c, px, py);
        int oos = 0;
        for (int k = 0; k < 4; ++k)
            if (px[k] < -100.0f || px[k] > (float)W + 100.0f || py[k] < -100.0f || py[k] > (float)H + 100.0f) oos = 1;
        if (oos) { done[i] = 1; status[i] = ST_CRASH_WALL; continue; }
        int off = 0;
        for (int k = 0; k < 4; ++k)
            if (!on_road(e, px[k], py[k])) off = 1;
        if (off) { done[i] = 1; status[i] = ST_CRASH_WALL; continue; }
        int line = 0;
        for (int k = 0; k < 4; ++k)
            if (yellow(e, px[k], py[k])) line = 1;
        if (!line)
            for (int k = 0; k < 4; ++k) {
                int k2 = (k + 1) & 3;
                float mx = 0.5f * (px[k] + px[k2]), my = 0.5f * (py[k] + py[k2]);
                if (is_line(e, (int)mx, (int)my)) line = 1;
            }
        if (!line)
            for (int k = 0; k < 4; ++k)
                if (is_line(e, (int)px[k], (int)py[k])) line = 1;
        if (line) { done[i] = 1; status[i] = ST_CRASH_LINE; }
    }
    for (int i = 0; i < n; ++i) { /* car-car, :292-318 */
        if (!e->ego[i].alive || done[i]) continue;
        for (int j = i + 1; j < n; ++j) {
            if (!e->ego[j].alive || done[j]) continue;
            if (collide(&e->ego[i], &e->ego[j])) {
                done[i] = done[j] = 1;
                status[i] = status[j] = ST_CRASH_CAR;
            }
        }
        if (e->traffic)
            for (int j = 0; j < e->nnpc; ++j) {
                if (!e->npc[j].alive) continue;
                if (collide(&e->ego[i], &e->npc[j])) { done[i] = 1; status[i] = ST_CRASH_CAR; break; }
            }
    }
    for (int i = 0; i < n; ++i) { /* bonuses, :320-326 */
        if (!done[i]) continue;
        if (status[i] == ST_CRASH_CAR) rew[i] += e->rc[3];
        else if (status[i] == ST_CRASH_WALL || status[i] == ST_CRASH_LINE) rew[i] += e->rc[4];
        else if (status[i] == ST_SUCCESS) rew[i] += e->rc[5];
    }
    if (e->use_team && n > 0) { /* :329-336 */
        float avg = 0.0f;
        for (int i = 0; i < n; ++i) avg += rew[i];
        avg /= (float)n;
        for (int i = 0; i < n; ++i) rew[i] = (1.0f - e->rc[7]) * rew[i] + e->rc[7] * avg;
    }
    int terminated = 0, alive_cnt = 0;
    if (e->respawn) { /* :339-368 */
        for (int i = 0; i < n; ++i)
            if (e->ego[i].alive && done[i] &&
                (status[i] == ST_CRASH_CAR || status[i] == ST_CRASH_WALL || status[i] == ST_CRASH_LINE))
                respawn(&e->ego[i]);
        int succ = 0;
        for (int i = 0; i < n; ++i) {
            if (!e->ego[i].alive) continue;
            ++alive_cnt;
            if (done[i] && status[i] == ST_SUCCESS) ++succ;
        }
        if (succ > 0 && succ == alive_cnt) terminated = 1;
    } else {
        for (int i = 0; i < n; ++i)
            if (done[i]) { terminated = 1; break; }
        for (int i = 0; i < n; ++i) alive_cnt += e->ego[i].alive ? 1 : 0;
    }
    int truncated = e->max_steps > 0 && step_no >= e->max_steps;
    /* LiDAR after respawn, :374-388: obstacles = egos (+ NPCs in traffic mode) */
    orc_car all[2 * MAXCARS];
    int nall = 0;
    for (int i = 0; i < n; ++i) all[nall++] = e->ego[i];
    if (e->traffic)
        for (int j = 0; j < e->nnpc; ++j) all[nall++] = e->npc[j];
    for (int i = 0; i < n; ++i)
        if (e->ego[i].alive) lidar_update(e, &e->ego[i], e->traffic ? -1 : i, all, nall, e->lidar + i * e->rays);
    observe(e, obs);
    flags[0] = terminated; flags[1] = truncated; flags[2] = alive_cnt; flags[3] = step_no;
}

int orc_sizeof_car(void) { return (int)sizeof(orc_car); }

/* Port throughput for the cpu_baseline fallback: `threads` is decided by the
 * caller (one process/thread per call); steps x E_local envs of N agents with
 * uniform actions from a tiny LCG, auto-reset on terminated/truncated. */
double orc_bench(int n, int rays, int use_team, int steps, unsigned seed) {
    static const int map3[12][2] = {{1, 4}, {2, 8}, {3, 12}, {4, 7}, {5, 11}, {6, 3},
                                    {7, 10}, {8, 2}, {9, 6}, {10, 1}, {11, 5}, {12, 9}};
    const float rc[8] = {10.0f, 1.0f, -0.01f, -10.0f, -5.0f, 10.0f, -0.02f, 0.2f};
    orc_env* e = orc_create(3, n, rays, 360.0f, 250.0f, 4.0f, 0, use_team, 1, 2000, 0, 0.5f, rc, 0);
    int routes[MAXCARS];
    for (int i = 0; i < n; ++i) routes[i] = orc_route_id(e, map3[i % 12][0] - 1, 12 + map3[i % 12][1] - 1);
    orc_reset(e, routes);
    float* obs = (float*)malloc(sizeof(float) * (size_t)n * (size_t)e->obs_dim);
    float rew[MAXCARS], act[2 * MAXCARS];
    uint8_t done[MAXCARS], st[MAXCARS];
    int32_t fl[4];
    uint32_t s = seed * 2654435761u + 1u;
    long long cnt = 0;
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int t = 0; t < steps; ++t) {
        for (int i = 0; i < 2 * n; ++i) {
            s = s * 1664525u + 1013904223u;
            act[i] = (float)(s >> 8) * (2.0f / 16777216.0f) - 1.0f;
        }
        orc_step(e, act, 1.0f / 60.0f, -1, obs, rew, done, st, fl);
        cnt += n;
        if (fl[0] || fl[1]) orc_reset(e, routes);
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    free(obs);
    orc_destroy(e);
    double sec = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    return (double)cnt / sec;
}
