/*
 * artis_constants.h -- physical and numerical constants with the exact values of the reference
 * (reference constants.h:5-43, artisoptions_classic.h for MINPOP / NU_MIN_R / NU_MAX_R / TABLESIZE defaults).
 * Parity depends on using the same literals (e.g. the reference's PI = 3.1415926535987 is not M_PI).
 * Shared by the synthetic-model generator, the CPU oracle and the HIP engine.
 */
#ifndef ARTIS_CONSTANTS_H
#define ARTIS_CONSTANTS_H

#define ARTIS_CLIGHT 2.99792458e+10
#define ARTIS_CLIGHT_PROP ARTIS_CLIGHT
#define ARTIS_H 6.6260755e-27
#define ARTIS_MSUN 1.98855e+33
#define ARTIS_LSUN 3.826e+33
#define ARTIS_MH 1.67352e-24
#define ARTIS_ME 9.1093897e-28
#define ARTIS_QE 4.80325E-10
#define ARTIS_PI 3.1415926535987
#define ARTIS_GREY_OP 0.1 /* globals.h:266 GREY_OP [cm^2/g] */
#define ARTIS_EV 1.6021772e-12
#define ARTIS_MEV 1.6021772e-6
#define ARTIS_DAY 86400.0
#define ARTIS_SIGMA_T 6.6524e-25
#define ARTIS_THOMSON_LIMIT 1e-2 /* constants.h:19 */
#define ARTIS_PARSEC 3.0857e+18
#define ARTIS_KB 1.38064852e-16
#define ARTIS_SAHACONST 2.0706659e-16

#define ARTIS_CLIGHTSQUARED 8.9875518e+20
#define ARTIS_TWOOVERCLIGHTSQUARED 2.2253001e-21
#define ARTIS_TWOHOVERCLIGHTSQUARED 1.4745007e-47
#define ARTIS_CLIGHTSQUAREDOVERTWOH 6.7819570e+46
#define ARTIS_ONEOVERH 1.509188961e+26
#define ARTIS_HOVERKB 4.799243681748932e-11
#define ARTIS_FOURPI 1.256637061600000e+01
#define ARTIS_ONEOVER4PI 7.957747153555701e-02
#define ARTIS_STEBO 5.670400e-5  /* constants.h:22 */
#define ARTIS_HCLIGHTOVERFOURPI 1.580764662876770e-17
#define ARTIS_OSCSTRENGTHCONVERSION 1.3473837e+21
#define ARTIS_H_IONPOT (13.5979996 * ARTIS_EV)
#define ARTIS_C_0 5.465e-11

/* artisoptions_classic.h values used by the hot path */
#define ARTIS_MINPOP 1e-30
#define ARTIS_NU_MIN_R 1e14
#define ARTIS_NU_MAX_R 5e15

/* kpkt.cc:18-23 cooling channel types */
#define ARTIS_COOLINGTYPE_FF 880
#define ARTIS_COOLINGTYPE_FB 881
#define ARTIS_COOLINGTYPE_COLLEXC 882
#define ARTIS_COOLINGTYPE_COLLION 883

/* rpkt.h event types */
#define ARTIS_RPKT_EVENTTYPE_BB 550
#define ARTIS_RPKT_EVENTTYPE_CONT 551

/* macroatom.h:6-27 */
#define ARTIS_MA_ACTION_RADDEEXC 0
#define ARTIS_MA_ACTION_COLDEEXC 1
#define ARTIS_MA_ACTION_RADRECOMB 2
#define ARTIS_MA_ACTION_COLRECOMB 3
#define ARTIS_MA_ACTION_INTERNALDOWNSAME 4
#define ARTIS_MA_ACTION_INTERNALDOWNLOWER 5
#define ARTIS_MA_ACTION_INTERNALUPSAME 6
#define ARTIS_MA_ACTION_INTERNALUPHIGHER 7
#define ARTIS_MA_ACTION_INTERNALUPHIGHERNT 8
#define ARTIS_MA_ACTION_COUNT 9

/* decay.h:15-22 */
#define ARTIS_DECAYTYPE_ALPHA 0
#define ARTIS_DECAYTYPE_ELECTRONCAPTURE 1
#define ARTIS_DECAYTYPE_BETAPLUS 2
#define ARTIS_DECAYTYPE_BETAMINUS 3
#define ARTIS_DECAYTYPE_NONE 4

/* stats.h:49-83 event counters */
enum artis_counter {
  CTR_MA_STAT_ACTIVATION_COLLEXC = 0,
  CTR_MA_STAT_ACTIVATION_COLLION = 1,
  CTR_MA_STAT_ACTIVATION_NTCOLLEXC = 2,
  CTR_MA_STAT_ACTIVATION_NTCOLLION = 3,
  CTR_MA_STAT_ACTIVATION_BB = 4,
  CTR_MA_STAT_ACTIVATION_BF = 5,
  CTR_MA_STAT_ACTIVATION_FB = 6,
  CTR_MA_STAT_DEACTIVATION_COLLDEEXC = 7,
  CTR_MA_STAT_DEACTIVATION_COLLRECOMB = 8,
  CTR_MA_STAT_DEACTIVATION_BB = 9,
  CTR_MA_STAT_DEACTIVATION_FB = 10,
  CTR_MA_STAT_INTERNALUPHIGHER = 11,
  CTR_MA_STAT_INTERNALUPHIGHERNT = 12,
  CTR_MA_STAT_INTERNALDOWNLOWER = 13,
  CTR_K_STAT_TO_MA_COLLEXC = 14,
  CTR_K_STAT_TO_MA_COLLION = 15,
  CTR_K_STAT_TO_R_FF = 16,
  CTR_K_STAT_TO_R_FB = 17,
  CTR_K_STAT_TO_R_BB = 18,
  CTR_K_STAT_FROM_FF = 19,
  CTR_K_STAT_FROM_BF = 20,
  CTR_NT_STAT_FROM_GAMMA = 21,
  CTR_NT_STAT_TO_IONIZATION = 22,
  CTR_NT_STAT_TO_EXCITATION = 23,
  CTR_NT_STAT_TO_KPKT = 24,
  CTR_K_STAT_FROM_EARLIERDECAY = 25,
  CTR_ESCOUNTER = 26,
  CTR_RESONANCESCATTERINGS = 27,
  CTR_CELLCROSSINGS = 28,
  CTR_UPSCATTER = 29,
  CTR_DOWNSCATTER = 30,
  CTR_UPDATECELL = 31,
  CTR_COOLINGRATECALCCOUNTER = 32,
  CTR_NESC = 33,
};

/* Work counters reported per call (artis_gpu_last_work_counts); they feed the algorithmic byte model of
 * SURVEY.md §8(d). Same meaning in oracle and engine. */
enum artis_work {
  WK_PACKETS_ACTIVE = 0,   /* packets not escaped and prop_time < t2 at call start */
  WK_RPKT_STEPS = 1,       /* do_rpkt_step calls */
  WK_LINES_SCANNED = 2,    /* get_event loop iterations with a reachable line */
  WK_LINE_TAUS = 3,        /* Sobolev tau evaluations */
  WK_KAPPA_EVALS = 4,      /* calculate_kappa_rpkt_cont evaluations */
  WK_BF_ACTIVE = 5,        /* continua summed over all kappa evaluations (nu >= nu_edge) */
  WK_EST_SEGMENTS = 6,     /* update_estimators calls in non-empty cells */
  WK_GC_UPDATES = 7,       /* gamma/bfheating estimator updates */
  WK_MA_JUMPS = 8,         /* macro-atom loop iterations */
  WK_MA_TRANS = 9,         /* transitions whose rates were evaluated in the macro-atom */
  WK_KPKT = 10,            /* k-packet conversions */
  WK_KPKT_TERMS = 11,      /* cooling terms scanned */
  WK_ESCAPED = 12,
  WK_ES_SCAT = 13,
  WK_BB_EVENTS = 14,
  WK_CONT_EVENTS = 15,
};

#endif /* ARTIS_CONSTANTS_H */
