// artis_io.cc -- the reference's packet and virtual-packet file formats (include/artis_io.h).
#include "artis_io.h"

#include <cmath>
#include <cstdio>
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

}  // namespace

extern "C" {

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
