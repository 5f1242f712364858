# Patch for tools/mkvar.sh (file ba_kernels.hip): k_jacobian with the X /
# scale gathers issued two chunks ahead instead of one (A/B variant).
def _rep(s, old, new):
    assert s.count(old) == 1, "patch_jac2: anchor not found:\n" + old
    return s.replace(old, new)
s = _rep(s, '''  int p_nxt = 0;                              // point index of chunk t + 1
  double2 uv_cur = make_double2(0.0, 0.0);    // chunk t
  double Xc[3] = {0.0, 0.0, 1.0}, spc[3] = {1.0, 1.0, 1.0};
  if (t < n_chunks) {
    const int64_t i = int64_t(chunks[t].y) + l;
    const int p0 = cm_p[i];
    uv_cur = ld2(uv_cm + 2 * i);
    p_nxt = cm_p[int64_t(chunk_at(t + 1).y) + l];
#pragma unroll
    for (int j = 0; j < 3; ++j) Xc[j] = X[3 * size_t(p0) + j];
    if (scaled)
#pragma unroll
      for (int j = 0; j < 3; ++j) spc[j] = scale_p[3 * size_t(p0) + j];
  }''', '''  int p_nxt = 0;                              // point index of chunk t + 2
  double2 uv_cur = make_double2(0.0, 0.0);    // chunk t
  double Xc[3] = {0.0, 0.0, 1.0}, spc[3] = {1.0, 1.0, 1.0};
  double Xn[3] = {0.0, 0.0, 1.0}, spn[3] = {1.0, 1.0, 1.0};  // chunk t + 1 (in flight)
  if (t < n_chunks) {
    const int64_t i = int64_t(chunks[t].y) + l;
    const int p0 = cm_p[i];
    const int p1 = cm_p[int64_t(chunk_at(t + 1).y) + l];
    uv_cur = ld2(uv_cm + 2 * i);
    p_nxt = cm_p[int64_t(chunk_at(t + 2).y) + l];
#pragma unroll
    for (int j = 0; j < 3; ++j) { Xc[j] = X[3 * size_t(p0) + j]; Xn[j] = X[3 * size_t(p1) + j]; }
    if (scaled)
#pragma unroll
      for (int j = 0; j < 3; ++j) { spc[j] = scale_p[3 * size_t(p0) + j]; spn[j] = scale_p[3 * size_t(p1) + j]; }
  }''')
s = _rep(s, '''  asm volatile("" : "+v"(Xc[0]), "+v"(Xc[1]), "+v"(Xc[2]), "+v"(spc[0]), "+v"(spc[1]), "+v"(spc[2]), "+v"(uv_cur.x),
               "+v"(uv_cur.y), "+v"(p_nxt));''', '''  asm volatile("" : "+v"(Xc[0]), "+v"(Xc[1]), "+v"(Xc[2]), "+v"(spc[0]), "+v"(spc[1]), "+v"(spc[2]), "+v"(uv_cur.x),
               "+v"(uv_cur.y), "+v"(p_nxt), "+v"(Xn[0]), "+v"(Xn[1]), "+v"(Xn[2]), "+v"(spn[0]), "+v"(spn[1]),
               "+v"(spn[2]));''')
s = _rep(s, '''    double Xn[3], spn[3] = {1.0, 1.0, 1.0};
#pragma unroll
    for (int j = 0; j < 3; ++j) Xn[j] = X[3 * size_t(p_nxt) + j];
    if (scaled)
#pragma unroll
      for (int j = 0; j < 3; ++j) spn[j] = scale_p[3 * size_t(p_nxt) + j];
    const int4 ch_n = chunk_at(t + 1);
    const double2 uv_nxt = ld2(uv_cm + 2 * (int64_t(ch_n.y) + l));
    const int p_nn = cm_p[int64_t(chunk_at(t + 2).y) + l];''', '''    double X2[3], sp2[3] = {1.0, 1.0, 1.0};
#pragma unroll
    for (int j = 0; j < 3; ++j) X2[j] = X[3 * size_t(p_nxt) + j];
    if (scaled)
#pragma unroll
      for (int j = 0; j < 3; ++j) sp2[j] = scale_p[3 * size_t(p_nxt) + j];
    const int4 ch_n = chunk_at(t + 1);
    const double2 uv_nxt = ld2(uv_cm + 2 * (int64_t(ch_n.y) + l));
    const int p_nn = cm_p[int64_t(chunk_at(t + 3).y) + l];''')
s = _rep(s, '''    for (int j = 0; j < 3; ++j) { Xc[j] = Xn[j]; spc[j] = spn[j]; }
    uv_cur = uv_nxt;
    p_nxt = p_nn;''', '''    for (int j = 0; j < 3; ++j) { Xc[j] = Xn[j]; spc[j] = spn[j]; Xn[j] = X2[j]; spn[j] = sp2[j]; }
    uv_cur = uv_nxt;
    p_nxt = p_nn;''')
