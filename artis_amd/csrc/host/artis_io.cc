// artis_io.cc -- the reference's packet and virtual-packet file formats (include/artis_io.h).
#include "artis_io.h"

#include "artis_constants.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

namespace {

constexpr double kDay = 86400.0;

struct File {
  FILE *f;
  explicit File(const char *path, const char *mode) : f(path ? std::fopen(path, mode) : nullptr) {}
  ~File() {
    if (f) std::fclose(f);
  }
};

// init_vspecpol (vpkt.cc:425-436): float lower_time / delta_t and lower_freq_vspec / delta_freq_vspec
void vspec_bins(const artis_vpkt_params *p, std::vector<float> &lt, std::vector<float> &dt, std::vector<float> &lf,
                std::vector<float> &df) {
  const double dlogt = (log(p->tmax_vspec) - log(p->tmin_vspec)) / p->vmtbins;
  const double dlognu = (log(p->numax_vspec) - log(p->numin_vspec)) / p->vmnubins;
  lt.resize(p->vmtbins);
  dt.resize(p->vmtbins);
  for (int n = 0; n < p->vmtbins; n++) {
    lt[n] = (float)exp(log(p->tmin_vspec) + (n * (dlogt)));
    dt[n] = (float)(exp(log(p->tmin_vspec) + ((n + 1) * (dlogt))) - lt[n]);
  }
  lf.resize(p->vmnubins);
  df.resize(p->vmnubins);
  for (int m = 0; m < p->vmnubins; m++) {
    lf[m] = (float)exp(log(p->numin_vspec) + (m * (dlognu)));
    df[m] = (float)(exp(log(p->numin_vspec) + ((m + 1) * (dlognu))) - lf[m]);
  }
}

bool line_is_comment_only(const std::string &line) {  // lineiscommentonly (sn3d.h)
  for (char ch : line) {
    if (ch == '#') return true;
    if (ch != ' ' && ch != '\t') return false;
  }
  return true;
}

std::string temp_packets_name(const char *dir, int timestep, int my_rank) {
  char name[128];
  std::snprintf(name, sizeof name, "packets_%.4d_ts%d.tmp", my_rank, timestep);
  return (dir && dir[0]) ? std::string(dir) + "/" + name : std::string(name);
}

// input.h:16-30 lineiscommentonly: blank up to an optional '#' (only ' ' counts as blank)
bool ref_comment_only(const std::string &line) {
  size_t n = line.find('#');
  if (n == std::string::npos) n = line.length();
  for (size_t i = 0; i < n; i++)
    if (line[i] != ' ') return false;
  return true;
}

// input.cc:1833-1846 get_noncommentline
bool noncomment_line(std::istream &in, std::string &line) {
  while (std::getline(in, line))
    if (!ref_comment_only(line)) return true;
  return false;
}

// grid.cc:1080-1156 read_model_headerline: the number of custom columns after the standard ones, with the
// reference's column-position checks
bool model_header_columns(const std::string &line, int model_type, int *ncustom) {
  std::istringstream iss(line);
  std::string token;
  int columnindex = -1;
  *ncustom = 0;
  while (std::getline(iss, token, ' ')) {
    bool blank = true;
    for (char ch : token)
      if (!isspace((unsigned char)ch)) blank = false;
    if (blank) continue;
    columnindex++;
    if (token == "#inputcellid") {
      if (columnindex != 0) return false;
    } else if (token == "velocity_outer") {
      if (columnindex != 1) return false;
    } else if (token == "logrho") {
      if (columnindex != 2 || model_type != 1) return false;
    } else if (token == "rho") {
      if (columnindex != 4 || model_type == 1) return false;
    } else if (token == "X_Fegroup" || token == "X_Ni56" || token == "X_Co56" || token == "X_Fe52" ||
               token == "X_Cr48" || token == "X_Ni57" || token == "X_Co57" || token.rfind("pos_", 0) == 0) {
      continue;
    } else {
      if (model_type == 1 && columnindex < 10) return false;
      if (model_type == 3 && columnindex < 12) return false;
      (*ncustom)++;
    }
  }
  return true;
}

void alloc_model_arrays(artis_ejecta_model *m, int n) {
  double **arrs[8] = {&m->rho_model, &m->ffegrp, &m->x_ni56, &m->x_co56, &m->x_fe52, &m->x_cr48, &m->x_ni57,
                      &m->x_co57};
  for (double **a : arrs) *a = (double *)std::calloc((size_t)n, sizeof(double));
}

// read_2d3d_modelradioabundanceline (grid.cc:1158-1226): 5 or 7 abundances, then with 7 the custom columns
bool model_abundance_line(const std::string &line, artis_ejecta_model *m, int mgi, bool keepcell) {
  double v[7] = {0, 0, 0, 0, 0, 0, 0};
  const int items = std::sscanf(line.c_str(), "%lg %lg %lg %lg %lg %lg %lg", &v[0], &v[1], &v[2], &v[3], &v[4],
                                &v[5], &v[6]);
  if (items != 5 && items != 7) return false;
  if (keepcell) {
    m->ffegrp[mgi] = v[0];
    m->x_ni56[mgi] = v[1];
    m->x_co56[mgi] = v[2];
    m->x_fe52[mgi] = v[3];
    m->x_cr48[mgi] = v[4];
    m->x_ni57[mgi] = v[5];
    m->x_co57[mgi] = v[6];
    if (items == 7) {
      std::istringstream ss(line);
      double x;
      for (int i = 0; i < 7 + m->n_custom_columns; i++)
        if (!(ss >> x)) return false;
      if (ss >> x) return false;  // no tokens left (grid.cc:1217-1218)
    }
  }
  return true;
}

}  // namespace

extern "C" {

// input.cc:1874-2140 read_parameterfile
int artis_read_input_file(const char *filename, artis_input_params *p) {
  if (!filename || !p) return ARTIS_ERR_BAD_ARGUMENT;
  std::ifstream in(filename);
  if (!in.is_open()) return ARTIS_ERR_BAD_ARGUMENT;
  std::memset(p, 0, sizeof(*p));
  std::string line;
  auto next = [&](std::istringstream &ss) {
    if (!noncomment_line(in, line)) return false;
    ss.clear();
    ss.str(line);
    return true;
  };
  std::istringstream ss;
  long dum1 = 0;
  float dum2 = 0.f, dum3 = 0.f;
  if (!next(ss) || !(ss >> dum1)) return ARTIS_ERR_BAD_ARGUMENT;
  p->pre_zseed = dum1 > 0 ? (uint32_t)dum1 : 0u;
  if (!next(ss) || !(ss >> p->ntstep) || p->ntstep <= 0) return ARTIS_ERR_BAD_ARGUMENT;
  if (!next(ss) || !(ss >> p->itstep >> p->ftstep)) return ARTIS_ERR_BAD_ARGUMENT;
  if (!(p->itstep < p->ntstep && p->itstep <= p->ftstep && p->ftstep <= p->ntstep)) return ARTIS_ERR_BAD_ARGUMENT;
  if (!next(ss) || !(ss >> p->tmin_days >> p->tmax_days)) return ARTIS_ERR_BAD_ARGUMENT;
  if (!(p->tmin_days > 0 && p->tmax_days > 0 && p->tmin_days < p->tmax_days)) return ARTIS_ERR_BAD_ARGUMENT;
  if (!next(ss) || !(ss >> dum2 >> dum3)) return ARTIS_ERR_BAD_ARGUMENT;
  p->nusyn_min_mev = dum2;
  p->nusyn_max_mev = dum3;
  if (!next(ss) || !(ss >> p->nsyn_time)) return ARTIS_ERR_BAD_ARGUMENT;
  if (!next(ss) || !(ss >> dum2 >> dum3)) return ARTIS_ERR_BAD_ARGUMENT;
  p->syn_time_start_days = dum2;
  p->syn_time_dlog = dum3;
  if (!next(ss) || !(ss >> p->model_type)) return ARTIS_ERR_BAD_ARGUMENT;
  if (!next(ss) || !(ss >> p->rlc_mode) || p->rlc_mode < 0 || p->rlc_mode > 4) return ARTIS_ERR_BAD_ARGUMENT;
  p->do_r_lc = (p->rlc_mode != 0);
  p->do_rlc_est = (p->rlc_mode > 0) ? p->rlc_mode - 1 : 0;
  if (!next(ss) || !(ss >> p->n_out_it)) return ARTIS_ERR_BAD_ARGUMENT;
  if (!next(ss) || !(ss >> dum2) || std::fabs(dum2 - 1.) >= 1e-3) return ARTIS_ERR_BAD_ARGUMENT;
  p->clight_factor = dum2;
  if (!next(ss) || !(ss >> p->gamma_grey)) return ARTIS_ERR_BAD_ARGUMENT;
  float sd[3] = {0.f, 0.f, 0.f};
  if (!next(ss) || !(ss >> sd[0] >> sd[1] >> sd[2])) return ARTIS_ERR_BAD_ARGUMENT;
  const double rr = (sd[0] * sd[0]) + (sd[1] * sd[1]) + (sd[2] * sd[2]);
  for (int d = 0; d < 3; d++) p->syn_dir[d] = rr > 1.e-6 ? sd[d] / sqrt(rr) : 0.;
  if (!next(ss) || !(ss >> p->opacity_case)) return ARTIS_ERR_BAD_ARGUMENT;
  if (!next(ss) || !(ss >> p->rho_crit_para)) return ARTIS_ERR_BAD_ARGUMENT;
  if (!next(ss) || !(ss >> p->debug_packet)) return ARTIS_ERR_BAD_ARGUMENT;
  if (!next(ss) || !(ss >> p->continued_from_saved)) return ARTIS_ERR_BAD_ARGUMENT;
  p->continued_from_saved = (p->continued_from_saved == 1);
  if (!p->continued_from_saved && p->itstep != 0) return ARTIS_ERR_BAD_ARGUMENT;  // input.cc:2033
  if (!next(ss) || !(ss >> dum2)) return ARTIS_ERR_BAD_ARGUMENT;
  p->rfcut_angstroms = dum2;
  if (!next(ss) || !(ss >> p->num_lte_timesteps)) return ARTIS_ERR_BAD_ARGUMENT;
  if (!next(ss) || !(ss >> p->cell_is_optically_thick >> p->num_grey_timesteps)) return ARTIS_ERR_BAD_ARGUMENT;
  if (!next(ss) || !(ss >> p->max_bf_continua)) return ARTIS_ERR_BAD_ARGUMENT;
  if (p->max_bf_continua == -1) p->max_bf_continua = 1000000;
  if (!next(ss) || !(ss >> p->nprocs_exspec)) return ARTIS_ERR_BAD_ARGUMENT;
  if (!next(ss) || !(ss >> p->do_emission_res)) return ARTIS_ERR_BAD_ARGUMENT;
  float kts = 0.f;
  if (!next(ss) || !(ss >> kts >> p->n_kpktdiffusion_timesteps)) return ARTIS_ERR_BAD_ARGUMENT;
  p->kpktdiffusion_timescale = kts;
  return 0;
}

void artis_free_model(artis_ejecta_model *m) {
  if (!m) return;
  double *arrs[9] = {m->vout, m->rho_model, m->ffegrp, m->x_ni56, m->x_co56, m->x_fe52, m->x_cr48, m->x_ni57,
                     m->x_co57};
  for (double *a : arrs) std::free(a);
  std::free(m->pos_model);
  std::memset(m, 0, sizeof(*m));
}

// grid.cc:1228-1370 (1D) and 1459-1600 (3D)
int artis_read_model(const char *filename, int model_type, artis_ejecta_model *m) {
  if (!filename || !m || (model_type != 1 && model_type != 3)) return ARTIS_ERR_BAD_ARGUMENT;
  std::memset(m, 0, sizeof(*m));
  std::ifstream in(filename);
  if (!in.is_open()) return ARTIS_ERR_BAD_ARGUMENT;
  m->model_type = model_type;
  std::string line;
  int npts = 0;
  if (!noncomment_line(in, line) || !(std::stringstream(line) >> npts) || npts <= 0) return ARTIS_ERR_BAD_ARGUMENT;
  m->npts_model = npts;
  double t_model_days = 0.;
  if (!noncomment_line(in, line) || !(std::stringstream(line) >> t_model_days)) return ARTIS_ERR_BAD_ARGUMENT;
  m->t_model = t_model_days * kDay;
  if (model_type == 3) {
    const int n = (int)std::lround(std::pow(npts, 1 / 3.));
    if (n * n * n != npts) return ARTIS_ERR_BAD_ARGUMENT;  // grid.cc:1475-1476
    m->ncoord_model[0] = m->ncoord_model[1] = m->ncoord_model[2] = n;
    if (!noncomment_line(in, line) || !(std::stringstream(line) >> m->vmax)) return ARTIS_ERR_BAD_ARGUMENT;
  } else {
    m->ncoord_model[0] = npts;
    m->ncoord_model[1] = m->ncoord_model[2] = 1;
  }
  // optional custom header line (grid.cc:1262-1268)
  std::streampos oldpos = in.tellg();
  if (std::getline(in, line) && ref_comment_only(line)) {
    if (!model_header_columns(line, model_type, &m->n_custom_columns)) return ARTIS_ERR_BAD_ARGUMENT;
  } else {
    in.clear();
    in.seekg(oldpos);
  }
  alloc_model_arrays(m, npts);
  int rc = 0;
  int mgi = 0;
  if (model_type == 1) {
    m->vout = (double *)std::calloc((size_t)npts, sizeof(double));
    while (rc == 0 && mgi < npts && std::getline(in, line)) {
      int cellnumberin = 0;
      double vout_kmps = 0, log_rho = 0, v[7] = {0, 0, 0, 0, 0, 0, 0};
      const int items = std::sscanf(line.c_str(), "%d %lg %lg %lg %lg %lg %lg %lg %lg %lg", &cellnumberin, &vout_kmps,
                                    &log_rho, &v[0], &v[1], &v[2], &v[3], &v[4], &v[5], &v[6]);
      if ((items != 8 && items != 10) || cellnumberin != mgi + 1) {
        rc = ARTIS_ERR_BAD_ARGUMENT;
        break;
      }
      m->vout[mgi] = vout_kmps * 1.e5;
      m->rho_model[mgi] = std::pow(10., log_rho);
      m->ffegrp[mgi] = v[0];
      m->x_ni56[mgi] = v[1];
      m->x_co56[mgi] = v[2];
      m->x_fe52[mgi] = v[3];
      m->x_cr48[mgi] = v[4];
      m->x_ni57[mgi] = v[5];
      m->x_co57[mgi] = v[6];
      if (items == 10) {  // custom columns follow, and nothing after them (grid.cc:1328-1354)
        std::istringstream ss(line);
        double x;
        for (int i = 0; i < 10 + m->n_custom_columns; i++)
          if (!(ss >> x)) rc = ARTIS_ERR_BAD_ARGUMENT;
        if (ss >> x) rc = ARTIS_ERR_BAD_ARGUMENT;
      }
      mgi++;
    }
    if (rc == 0 && mgi == npts) m->vmax = m->vout[npts - 1];
  } else {
    m->pos_model = (float *)std::calloc((size_t)npts * 3, sizeof(float));
    const double xmax_tmodel = m->vmax * m->t_model;
    const int n = m->ncoord_model[0];
    bool posmatch_xyz = true, posmatch_zyx = true;
    while (rc == 0 && mgi < npts && std::getline(in, line)) {
      int mgi_in = 0;
      float pos[3] = {0, 0, 0}, rho = 0;
      if (std::sscanf(line.c_str(), "%d %g %g %g %g", &mgi_in, &pos[0], &pos[1], &pos[2], &rho) != 5 ||
          mgi_in != mgi + 1 || rho < 0) {
        rc = ARTIS_ERR_BAD_ARGUMENT;
        break;
      }
      const int coord[3] = {mgi % n, (mgi / n) % n, mgi / (n * n)};  // get_cellcoordpointnum (grid.cc:172-199)
      for (int axis = 0; axis < 3; axis++) {
        const double cellwidth = 2 * xmax_tmodel / n;
        const double expected = -xmax_tmodel + cellwidth * coord[axis];
        if (std::fabs(expected - pos[axis]) > 0.5 * cellwidth) posmatch_xyz = false;
        if (std::fabs(expected - pos[2 - axis]) > 0.5 * cellwidth) posmatch_zyx = false;
        m->pos_model[(size_t)mgi * 3 + axis] = pos[axis];
      }
      m->rho_model[mgi] = rho;
      if (!std::getline(in, line) || !model_abundance_line(line, m, mgi, rho > 0)) {
        rc = ARTIS_ERR_BAD_ARGUMENT;
        break;
      }
      mgi++;
    }
    if (rc == 0 && !(posmatch_xyz ^ posmatch_zyx)) rc = ARTIS_ERR_BAD_ARGUMENT;  // grid.cc:1586
    m->posorder_zyx = posmatch_zyx ? 1 : 0;
  }
  if (rc == 0 && mgi != npts) rc = ARTIS_ERR_BAD_ARGUMENT;
  if (rc) artis_free_model(m);
  return rc;
}

// grid.cc:1007-1073 abundances_read
int artis_read_abundances(const char *filename, int npts_model, int model_type, int nelements,
                          const int32_t *anumber, float *elem_abund) {
  if (!filename || npts_model <= 0 || nelements < 0 || (nelements > 0 && (!anumber || !elem_abund)))
    return ARTIS_ERR_BAD_ARGUMENT;
  std::ifstream in(filename);
  if (!in.is_open()) return ARTIS_ERR_BAD_ARGUMENT;
  std::string line;
  for (int mgi = 0; mgi < npts_model; mgi++) {
    if (!noncomment_line(in, line)) return ARTIS_ERR_BAD_ARGUMENT;
    std::istringstream ss(line);
    int cellnumberinput = -1;
    if (!(ss >> cellnumberinput) || cellnumberinput != mgi + 1) return ARTIS_ERR_BAD_ARGUMENT;
    double normfactor = 0.;
    float abundances_in[150] = {0.f};
    for (int z = 1; z <= 150; z++) {
      abundances_in[z - 1] = 0.;
      if (!(ss >> abundances_in[z - 1])) {
        if (z == 1) return ARTIS_ERR_BAD_ARGUMENT;  // at least hydrogen
        break;
      }
      if (abundances_in[z - 1] < 0.) return ARTIS_ERR_BAD_ARGUMENT;
      normfactor += abundances_in[z - 1];
    }
    if (model_type == 3 || normfactor <= 0.) normfactor = 1.;
    for (int e = 0; e < nelements; e++) {
      const int z = anumber[e];
      elem_abund[(size_t)mgi * nelements + e] = (z >= 1 && z <= 150) ? (float)(abundances_in[z - 1] / normfactor) : 0.f;
    }
  }
  return 0;
}

// packet.cc:152-196
int artis_write_packets(const char *filename, const artis_packet *pkt, int npkts) {
  File out(filename, "w");
  if (!out.f || npkts < 0 || (npkts > 0 && !pkt)) return ARTIS_ERR_BAD_ARGUMENT;
  FILE *f = out.f;
  std::fprintf(f,
               "#number where type_id posx posy posz dirx diry dirz last_cross tdecay e_cmf e_rf nu_cmf nu_rf "
               "escape_type_id escape_time scat_count next_trans interactions last_event emissiontype trueemissiontype "
               "em_posx em_posy em_posz absorption_type absorption_freq nscatterings em_time absorptiondirx "
               "absorptiondiry absorptiondirz stokes1 stokes2 stokes3 pol_dirx pol_diry pol_dirz "
               "originated_from_positron true_emission_velocity trueem_time pellet_nucindex\n");
  for (int i = 0; i < npkts; i++) {
    const artis_packet &p = pkt[i];
    std::fprintf(f, "%d ", p.number);
    std::fprintf(f, "%d ", p.where);
    std::fprintf(f, "%d ", p.type);
    std::fprintf(f, "%lg %lg %lg ", p.pos[0], p.pos[1], p.pos[2]);
    std::fprintf(f, "%lg %lg %lg ", p.dir[0], p.dir[1], p.dir[2]);
    std::fprintf(f, "%d ", p.last_cross);
    std::fprintf(f, "%g ", p.tdecay);
    std::fprintf(f, "%g ", p.e_cmf);
    std::fprintf(f, "%g ", p.e_rf);
    std::fprintf(f, "%g ", p.nu_cmf);
    std::fprintf(f, "%g ", p.nu_rf);
    std::fprintf(f, "%d ", p.escape_type);
    std::fprintf(f, "%d ", p.escape_time);
    std::fprintf(f, "%d ", p.scat_count);
    std::fprintf(f, "%d ", p.next_trans);
    std::fprintf(f, "%d ", p.interactions);
    std::fprintf(f, "%d ", p.last_event);
    std::fprintf(f, "%d ", p.emissiontype);
    std::fprintf(f, "%d ", p.trueemissiontype);
    std::fprintf(f, "%lg %lg %lg ", p.em_pos[0], p.em_pos[1], p.em_pos[2]);
    std::fprintf(f, "%d ", p.absorptiontype);
    std::fprintf(f, "%lg ", p.absorptionfreq);
    std::fprintf(f, "%d ", p.nscatterings);
    std::fprintf(f, "%d ", p.em_time);
    std::fprintf(f, "%lg %lg %lg ", p.absorptiondir[0], p.absorptiondir[1], p.absorptiondir[2]);
    std::fprintf(f, "%lg %lg %lg ", p.stokes[0], p.stokes[1], p.stokes[2]);
    std::fprintf(f, "%lg %lg %lg ", p.pol_dir[0], p.pol_dir[1], p.pol_dir[2]);
    std::fprintf(f, "%d ", (int)p.originated_from_particlenotgamma);
    std::fprintf(f, "%g ", p.trueemissionvelocity);
    std::fprintf(f, "%d ", p.trueem_time);
    std::fprintf(f, "%d ", p.pellet_nucindex);
    std::fprintf(f, "\n");
  }
  return std::ferror(f) ? ARTIS_ERR_BAD_ARGUMENT : 0;
}

// packet.cc:211-290 (the reference aborts on a short or long file; here that is the return code)
int artis_read_packets(const char *filename, artis_packet *pkt, int npkts) {
  if (!filename || npkts < 0 || (npkts > 0 && !pkt)) return ARTIS_ERR_BAD_ARGUMENT;
  std::ifstream in(filename);
  if (!in.is_open()) return ARTIS_ERR_BAD_ARGUMENT;
  std::string line;
  int packets_read = 0;
  while (std::getline(in, line)) {
    if (line_is_comment_only(line)) continue;
    packets_read++;
    const int i = packets_read - 1;
    if (i > npkts - 1) return ARTIS_ERR_BAD_ARGUMENT;
    artis_packet &p = pkt[i];
    std::istringstream s(line);
    int type_in = 0, last_cross_in = 0, escape_type = 0, origin = 0;
    s >> p.number >> p.where >> type_in;
    p.type = type_in;
    s >> p.pos[0] >> p.pos[1] >> p.pos[2];
    s >> p.dir[0] >> p.dir[1] >> p.dir[2];
    s >> last_cross_in;
    p.last_cross = last_cross_in;
    s >> p.tdecay;
    s >> p.e_cmf >> p.e_rf >> p.nu_cmf >> p.nu_rf;
    s >> escape_type >> p.escape_time >> p.scat_count;
    p.escape_type = escape_type;
    s >> p.next_trans >> p.interactions >> p.last_event;
    if (p.interactions < 0) return ARTIS_ERR_BAD_ARGUMENT;
    s >> p.emissiontype >> p.trueemissiontype;
    s >> p.em_pos[0] >> p.em_pos[1] >> p.em_pos[2];
    s >> p.absorptiontype >> p.absorptionfreq >> p.nscatterings;
    s >> p.em_time;
    s >> p.absorptiondir[0] >> p.absorptiondir[1] >> p.absorptiondir[2];
    s >> p.stokes[0] >> p.stokes[1] >> p.stokes[2];
    s >> p.pol_dir[0] >> p.pol_dir[1] >> p.pol_dir[2];
    s >> origin;
    p.originated_from_particlenotgamma = (origin != 0);
    s >> p.trueemissionvelocity;
    s >> p.trueem_time;
    s >> p.pellet_nucindex;
    if (s.fail()) return ARTIS_ERR_BAD_ARGUMENT;
  }
  return (packets_read < npkts) ? ARTIS_ERR_BAD_ARGUMENT : 0;
}

// sn3d.cc:387-398: raw fwrite of the 304-byte records
int artis_write_temp_packetsfile(const char *dir, int timestep, int my_rank, const artis_packet *pkts, int npkts) {
  if (npkts < 0 || (npkts > 0 && !pkts)) return ARTIS_ERR_BAD_ARGUMENT;
  const std::string path = temp_packets_name(dir, timestep, my_rank);
  File out(path.c_str(), "wb");
  if (!out.f) return ARTIS_ERR_BAD_ARGUMENT;
  if (std::fwrite(pkts, sizeof(artis_packet), npkts, out.f) != (size_t)npkts) return ARTIS_ERR_BAD_ARGUMENT;
  return 0;
}

// packet.cc:198-209
int artis_read_temp_packetsfile(const char *dir, int timestep, int my_rank, artis_packet *pkts, int npkts) {
  if (npkts < 0 || (npkts > 0 && !pkts)) return ARTIS_ERR_BAD_ARGUMENT;
  const std::string path = temp_packets_name(dir, timestep, my_rank);
  File in(path.c_str(), "rb");
  if (!in.f) return ARTIS_ERR_BAD_ARGUMENT;
  if (std::fread(pkts, sizeof(artis_packet), npkts, in.f) != (size_t)npkts) return ARTIS_ERR_BAD_ARGUMENT;
  return 0;
}

// vpkt.cc:445-483
int artis_write_vspecpol(const char *filename, const artis_vpkt_params *p, const artis_vpkt_result *r) {
  if (!p || !r || !r->vstokes_i || !r->vstokes_q || !r->vstokes_u || p->vmtbins <= 0 || p->vmnubins <= 0)
    return ARTIS_ERR_BAD_ARGUMENT;
  File out(filename, "w");
  if (!out.f) return ARTIS_ERR_BAD_ARGUMENT;
  FILE *f = out.f;
  std::vector<float> lt, dt, lf, df;
  vspec_bins(p, lt, dt, lf, df);
  const int ncomb = p->nobs * p->nspectra;
  const double *st[3] = {r->vstokes_i, r->vstokes_q, r->vstokes_u};
  for (int ind_comb = 0; ind_comb < ncomb; ind_comb++) {
    std::fprintf(f, "%g ", 0.);
    for (int l = 0; l < 3; l++)
      for (int t = 0; t < p->vmtbins; t++) std::fprintf(f, "%g ", (lt[t] + (dt[t] / 2.)) / kDay);
    std::fprintf(f, "\n");
    for (int m = 0; m < p->vmnubins; m++) {
      std::fprintf(f, "%g ", (lf[m] + (df[m] / 2.)));
      for (int l = 0; l < 3; l++)
        for (int t = 0; t < p->vmtbins; t++)
          std::fprintf(f, "%g ", st[l][((size_t)t * ncomb + ind_comb) * p->vmnubins + m]);
      std::fprintf(f, "\n");
    }
  }
  return std::ferror(f) ? ARTIS_ERR_BAD_ARGUMENT : 0;
}

// vpkt.cc:485-545 (the time / frequency columns are read and dropped, as the reference does)
int artis_read_vspecpol(const char *filename, const artis_vpkt_params *p, artis_vpkt_result *r) {
  if (!p || !r || !r->vstokes_i || !r->vstokes_q || !r->vstokes_u || p->vmtbins <= 0 || p->vmnubins <= 0)
    return ARTIS_ERR_BAD_ARGUMENT;
  File in(filename, "r");
  if (!in.f) return ARTIS_ERR_BAD_ARGUMENT;
  FILE *f = in.f;
  const int ncomb = p->nobs * p->nspectra;
  double *st[3] = {r->vstokes_i, r->vstokes_q, r->vstokes_u};
  float a = 0.f;
  for (int ind_comb = 0; ind_comb < ncomb; ind_comb++) {
    if (std::fscanf(f, "%g ", &a) != 1) return ARTIS_ERR_BAD_ARGUMENT;
    for (int l = 0; l < 3; l++)
      for (int t = 0; t < p->vmtbins; t++)
        if (std::fscanf(f, "%g ", &a) != 1) return ARTIS_ERR_BAD_ARGUMENT;
    for (int m = 0; m < p->vmnubins; m++) {
      if (std::fscanf(f, "%g ", &a) != 1) return ARTIS_ERR_BAD_ARGUMENT;
      for (int l = 0; l < 3; l++)
        for (int t = 0; t < p->vmtbins; t++)
          if (std::fscanf(f, "%lg ", &st[l][((size_t)t * ncomb + ind_comb) * p->vmnubins + m]) != 1)
            return ARTIS_ERR_BAD_ARGUMENT;
    }
  }
  return 0;
}

// vpkt.cc:629-646 with the yvel / zvel bin centres of init_vpkt_grid (vpkt.cc:548-574)
int artis_write_vpkt_grid(const char *filename, const artis_vpkt_params *p, double vmax, const artis_vpkt_result *r) {
  if (!p || !r || !r->vgrid_i || !r->vgrid_q || !r->vgrid_u || p->ny_vgrid <= 0 || p->nz_vgrid <= 0)
    return ARTIS_ERR_BAD_ARGUMENT;
  File out(filename, "w");
  if (!out.f) return ARTIS_ERR_BAD_ARGUMENT;
  FILE *f = out.f;
  const double ybin = 2 * vmax / p->ny_vgrid;
  const double zbin = 2 * vmax / p->nz_vgrid;
  for (int bin = 0; bin < p->nobs; bin++)
    for (int bin_range = 0; bin_range < p->nrange_grid; bin_range++)
      for (int n = 0; n < p->ny_vgrid; n++)
        for (int m = 0; m < p->nz_vgrid; m++) {
          const size_t idx = (((size_t)n * p->nz_vgrid + m) * p->nrange_grid + bin_range) * p->nobs + bin;
          std::fprintf(f, "%g ", vmax - (n + 0.5) * ybin);
          std::fprintf(f, "%g ", vmax - (m + 0.5) * zbin);
          std::fprintf(f, "%g ", r->vgrid_i[idx]);
          std::fprintf(f, "%g ", r->vgrid_q[idx]);
          std::fprintf(f, "%g ", r->vgrid_u[idx]);
          std::fprintf(f, "\n");
        }
  return std::ferror(f) ? ARTIS_ERR_BAD_ARGUMENT : 0;
}

// vpkt.cc:648-665
int artis_read_vpkt_grid(const char *filename, const artis_vpkt_params *p, artis_vpkt_result *r) {
  if (!p || !r || !r->vgrid_i || !r->vgrid_q || !r->vgrid_u || p->ny_vgrid <= 0 || p->nz_vgrid <= 0)
    return ARTIS_ERR_BAD_ARGUMENT;
  File in(filename, "r");
  if (!in.f) return ARTIS_ERR_BAD_ARGUMENT;
  FILE *f = in.f;
  double yv = 0., zv = 0.;
  for (int bin = 0; bin < p->nobs; bin++)
    for (int bin_range = 0; bin_range < p->nrange_grid; bin_range++)
      for (int n = 0; n < p->ny_vgrid; n++)
        for (int m = 0; m < p->nz_vgrid; m++) {
          const size_t idx = (((size_t)n * p->nz_vgrid + m) * p->nrange_grid + bin_range) * p->nobs + bin;
          if (std::fscanf(f, "%lg %lg %lg %lg %lg ", &yv, &zv, &r->vgrid_i[idx], &r->vgrid_q[idx], &r->vgrid_u[idx]) !=
              5)
            return ARTIS_ERR_BAD_ARGUMENT;
        }
  return 0;
}

}  // extern "C"

// ---- spectra / light curves (spectrum.cc:144-298, light_curve.cc:9-32) ------------------------------------------
namespace {
void spec_bins(int nnubins, double nu_min, double nu_max, std::vector<float> &lower, std::vector<float> &delta) {
  const double dlognu = (log(nu_max) - log(nu_min)) / nnubins;  // spectrum.cc:491-500
  lower.resize(nnubins);
  delta.resize(nnubins);
  for (int nnu = 0; nnu < nnubins; nnu++) {
    lower[nnu] = (float)exp(log(nu_min) + (nnu * (dlognu)));
    delta[nnu] = (float)(exp(log(nu_min) + ((nnu + 1) * (dlognu))) - lower[nnu]);
  }
}
struct FileCloser {
  FILE *f = nullptr;
  ~FileCloser() {
    if (f) fclose(f);
  }
};
constexpr double kLsun = 3.826e+33;
}  // namespace

int artis_write_spectrum(const char *spec_filename, const char *emission_filename, const char *trueemission_filename,
                         const char *absorption_filename, int ntstep, int numtimesteps, const double *ts_mid,
                         int nnubins, double nu_min, double nu_max, int proccount, int ioncount, const double *flux,
                         const double *emission, const double *trueemission, const double *absorption) {
  if (!spec_filename || !ts_mid || !flux || nnubins <= 0 || numtimesteps > ntstep || numtimesteps < 0) return -1;
  const bool do_emission_res = emission && trueemission && absorption && emission_filename && trueemission_filename &&
                               absorption_filename;
  FileCloser fs, fe, ft, fa;
  fs.f = fopen(spec_filename, "w");
  if (!fs.f) return -1;
  if (do_emission_res) {
    fe.f = fopen(emission_filename, "w");
    ft.f = fopen(trueemission_filename, "w");
    fa.f = fopen(absorption_filename, "w");
    if (!fe.f || !ft.f || !fa.f) return -1;
  }
  std::vector<float> lower, delta;
  spec_bins(nnubins, nu_min, nu_max, lower, delta);
  fprintf(fs.f, "%g ", 0.0);
  for (int p = 0; p < numtimesteps; p++) fprintf(fs.f, "%g ", ts_mid[p] / kDay);
  fprintf(fs.f, "\n");
  for (int nnu = 0; nnu < nnubins; nnu++) {
    fprintf(fs.f, "%g ", (lower[nnu] + (delta[nnu] / 2)));
    for (int nts = 0; nts < numtimesteps; nts++) {
      const size_t fi = (size_t)nts * nnubins + nnu;
      fprintf(fs.f, "%g ", flux[fi]);
      if (do_emission_res) {
        for (int i = 0; i < proccount; i++) fprintf(fe.f, "%g ", emission[fi * proccount + i]);
        fprintf(fe.f, "\n");
        for (int i = 0; i < proccount; i++) fprintf(ft.f, "%g ", trueemission[fi * proccount + i]);
        fprintf(ft.f, "\n");
        for (int i = 0; i < ioncount; i++) fprintf(fa.f, "%g ", absorption[fi * ioncount + i]);
        fprintf(fa.f, "\n");
      }
    }
    fprintf(fs.f, "\n");
  }
  return 0;
}

int artis_write_specpol(const char *specpol_filename, const char *emission_filename, const char *absorption_filename,
                        int ntstep, const double *ts_mid, int nnubins, double nu_min, double nu_max, int proccount,
                        int ioncount, const double *stokes_flux, const double *stokes_emission,
                        const double *stokes_absorption) {
  if (!specpol_filename || !ts_mid || !stokes_flux || nnubins <= 0 || ntstep <= 0) return -1;
  const bool do_emission_res = stokes_emission && stokes_absorption && emission_filename && absorption_filename;
  FileCloser fs, fe, fa;
  fs.f = fopen(specpol_filename, "w");
  if (!fs.f) return -1;
  if (do_emission_res) {
    fe.f = fopen(emission_filename, "w");
    fa.f = fopen(absorption_filename, "w");
    if (!fe.f || !fa.f) return -1;
  }
  std::vector<float> lower, delta;
  spec_bins(nnubins, nu_min, nu_max, lower, delta);
  fprintf(fs.f, "%g ", 0.0);
  for (int l = 0; l < 3; l++)
    for (int p = 0; p < ntstep; p++) fprintf(fs.f, "%g ", ts_mid[p] / kDay);
  fprintf(fs.f, "\n");
  const size_t nb = (size_t)ntstep * nnubins;
  for (int m = 0; m < nnubins; m++) {
    fprintf(fs.f, "%g ", (lower[m] + (delta[m] / 2)));
    for (int k = 0; k < 3; k++) {  // Stokes I, Q, U
      for (int p = 0; p < ntstep; p++) {
        const size_t fi = (size_t)p * nnubins + m;
        fprintf(fs.f, "%g ", stokes_flux[k * nb + fi]);
        if (do_emission_res) {
          for (int i = 0; i < proccount; i++) fprintf(fe.f, "%g ", stokes_emission[k * nb * proccount + fi * proccount + i]);
          fprintf(fe.f, "\n");
          for (int i = 0; i < ioncount; i++) fprintf(fa.f, "%g ", stokes_absorption[k * nb * ioncount + fi * ioncount + i]);
          fprintf(fa.f, "\n");
        }
      }
    }
    fprintf(fs.f, "\n");
  }
  return 0;
}

int artis_write_light_curve(const char *lc_filename, int abin, int numtimesteps, const double *ts_mid,
                            const double *ts_width, const double *lc_lum, const double *lc_lumcmf,
                            const double *gamma_dep, const double *cmf_lum) {
  if (!lc_filename || !ts_mid || !lc_lum || !lc_lumcmf || numtimesteps < 0) return -1;
  FileCloser f;
  f.f = fopen(lc_filename, "w");
  if (!f.f) return -1;
  for (int nts = 0; nts < numtimesteps; nts++)
    fprintf(f.f, "%g %g %g\n", ts_mid[nts] / kDay, (lc_lum[nts] / kLsun), (lc_lumcmf[nts] / kLsun));
  if (abin == -1) {
    for (int m = 0; m < numtimesteps; m++) {
      const double gd = gamma_dep ? gamma_dep[m] : 0., cl = cmf_lum ? cmf_lum[m] : 0.;
      fprintf(f.f, "%g %g %g\n", ts_mid[m] / kDay, (gd / kLsun / ts_width[m]), (cl / ts_width[m] / kLsun));
    }
  }
  return 0;
}

// ------------------------------------------------------------------------------------ Spencer-Fano input data
namespace {
struct NtStorage {
  std::vector<int32_t> Z, nelec, n, l;
  std::vector<double> ionpot_ev, A, B, C, D, prob, g_accumulated;
  std::vector<float> en_auger_ev, n_auger_elec_avg;
  std::vector<double> binding;
};
}  // namespace

int artis_read_nt_data(const char *dir, int nelements, const int32_t *anumber, const int32_t *ionstage0,
                       const int32_t *nions, int sfpts, double sf_emin, double sf_emax, artis_nt_data *out) {
  if (!dir || !out || nelements < 0 || (nelements > 0 && (!anumber || !ionstage0 || !nions)) || sfpts < 2 ||
      !(sf_emax > sf_emin) || !(sf_emin > 0.))
    return ARTIS_ERR_BAD_ARGUMENT;
  const int A1 = ARTIS_NT_MAX_AUGER + 1;
  auto path = [&](const char *name) { return std::string(dir) + "/" + name; };
  auto included = [&](int Z, int ionstage) {  // get_elementindex + the ion-stage range (nonthermal.cc:410-413)
    for (int e = 0; e < nelements; e++)
      if (anumber[e] == Z) return ionstage0[e] <= ionstage && ionstage < ionstage0[e] + nions[e];
    return false;
  };
  auto *st = new NtStorage();
  auto fail = [&]() {
    delete st;
    return ARTIS_ERR_BAD_ARGUMENT;
  };
  // read_binding_energies (nonthermal.cc:183-204): a 30 x 10 table in eV
  {
    File f(path("binding_energies.txt").c_str(), "r");
    int dum1 = 0, dum2 = 0;
    if (!f.f || std::fscanf(f.f, "%d %d", &dum1, &dum2) != 2 || dum1 != 10 || dum2 != 30) return fail();
    st->binding.assign(300, 0.);
    for (int i = 0; i < 30; i++)
      for (int j = 0; j < 10; j++) {
        float v = 0.f;
        if (std::fscanf(f.f, "%g", &v) != 1) return fail();
        st->binding[(size_t)i * 10 + j] = v * ARTIS_EV;
      }
  }
  // read_collion_data (nonthermal.cc:387-437)
  {
    File f(path("collion.txt").c_str(), "r");
    int count = 0;
    if (!f.f || std::fscanf(f.f, "%d", &count) != 1 || count < 0) return fail();
    for (int i = 0; i < count; i++) {
      int Z, nelec, n, l;
      double ip, A, B, C, D;
      if (std::fscanf(f.f, "%2d %2d %1d %1d %lg %lg %lg %lg %lg", &Z, &nelec, &n, &l, &ip, &A, &B, &C, &D) != 9)
        return fail();
      if (!included(Z, Z - nelec + 1)) continue;
      st->Z.push_back(Z);
      st->nelec.push_back(nelec);
      st->n.push_back(n);
      st->l.push_back(l);
      st->ionpot_ev.push_back(ip);
      st->A.push_back(A);
      st->B.push_back(B);
      st->C.push_back(C);
      st->D.push_back(D);
      for (int a = 0; a < A1; a++) st->prob.push_back(a == 0 ? 1. : 0.);
      st->g_accumulated.push_back(0.);
      st->en_auger_ev.push_back(0.f);
      st->n_auger_elec_avg.push_back(0.f);
    }
  }
  // read_auger_data (nonthermal.cc:255-385): fixed columns; X-ray subshells K L1 L2 L3 M1 M2 M3
  {
    File f(path("auger-km1993-table2.txt").c_str(), "r");
    if (!f.f) return fail();
    static const int xrayn[7] = {1, 2, 2, 2, 3, 3, 3}, xrayl[7] = {0, 0, 1, 1, 0, 1, 1}, xrayg[7] = {2, 2, 2, 4, 2, 2, 4};
    char line[151];
    while (std::fgets(line, 151, f.f)) {
      int Z = -1, ionstage = -1, offset = 0;
      if (std::sscanf(line, "%d %d%n", &Z, &ionstage, &offset) != 2 || offset != 5) return fail();
      if (!included(Z, ionstage)) continue;
      int shellnum = -1, epsilon_e3 = -1;
      float ionpot_ev = -1, en_total = -1;
      if (std::sscanf(line + 5, "%d %g %g %d%n", &shellnum, &ionpot_ev, &en_total, &epsilon_e3, &offset) != 4 ||
          offset != 20 || shellnum < 1 || shellnum > 7)
        return fail();
      float n_auger_elec_avg = 0;
      double prob[ARTIS_NT_MAX_AUGER + 1];
      for (int a = 0; a < 9; a++) {
        char strprob[6] = "00000";
        std::memcpy(strprob, line + 26 + a * 5, 5);
        strprob[5] = '\0';
        int probe4 = -1;
        if (std::sscanf(strprob, "%d", &probe4) != 1) return fail();
        const double p = probe4 / 10000.;
        if (!(p <= 1.0)) return fail();
        n_auger_elec_avg += a * p;
        if (a <= ARTIS_NT_MAX_AUGER)
          prob[a] = p;
        else
          prob[ARTIS_NT_MAX_AUGER] += p;
      }
      float en_auger_ev = en_total - (epsilon_e3 / 1000. * ionpot_ev);
      const int n = xrayn[shellnum - 1], l = xrayl[shellnum - 1], g = xrayg[shellnum - 1];
      if (!std::isfinite(en_auger_ev) || en_auger_ev < 0) en_auger_ev = 0.;
      for (size_t i = 0; i < st->Z.size(); i++) {
        if (st->Z[i] != Z || st->nelec[i] != Z - ionstage + 1 || st->n[i] != n || st->l[i] != l) continue;
        const double oldweight = st->g_accumulated[i] / (g + st->g_accumulated[i]);
        const double newweight = g / (g + st->g_accumulated[i]);
        st->g_accumulated[i] += g;
        st->en_auger_ev[i] = oldweight * st->en_auger_ev[i] + newweight * en_auger_ev;
        st->n_auger_elec_avg[i] = oldweight * st->n_auger_elec_avg[i] + newweight * n_auger_elec_avg;
        for (int a = 0; a < A1; a++) st->prob[i * A1 + a] = oldweight * st->prob[i * A1 + a] + newweight * prob[a];
      }
    }
  }
  artis_nt_shells &s = out->shells;
  std::memset(&s, 0, sizeof s);
  s.nshells = (int32_t)st->Z.size();
  s.sfpts = sfpts;
  s.sf_emin = sf_emin;
  s.sf_emax = sf_emax;
  s.Z = st->Z.data();
  s.nelec = st->nelec.data();
  s.n = st->n.data();
  s.l = st->l.data();
  s.ionpot_ev = st->ionpot_ev.data();
  s.A = st->A.data();
  s.B = st->B.data();
  s.C = st->C.data();
  s.D = st->D.data();
  s.prob_num_auger = st->prob.data();
  s.en_auger_ev = st->en_auger_ev.data();
  s.electron_binding = st->binding.data();
  out->storage = st;
  return 0;
}

void artis_free_nt_data(artis_nt_data *d) {
  if (!d) return;
  delete static_cast<NtStorage *>(d->storage);
  d->storage = nullptr;
  std::memset(&d->shells, 0, sizeof d->shells);
}
