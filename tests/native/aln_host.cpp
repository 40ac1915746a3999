// Host build of bwa mode's per-read logic (proovread_amd/csrc/aln_core.h, the code the
// device kernels run one lane per read) driven like pr_sw_launch drives the kernels: round 0
// extends every chain's first seed, the walk requests further seeds round by round, the
// final pass asks for mem_patch_reg scores in extra rounds.  Extensions come from the SW
// oracle (oracle/sw_oracle.c osw_extend_seed), so the CPU suite checks the walk, dedup,
// patch, primary and filter logic against oracle/aln_oracle.c without a GPU.
#include <cstring>
#include <vector>

#include "../../oracle/sw_oracle.h"
#include "../../proovread_amd/csrc/aln_core.h"

using namespace prgpu;

extern "C" int aln_host_run(const osw_opts *o, double drop_ratio, double mask_level, double mask_level_redun,
                            int max_chain_gap, int n_sr, const int64_t *sr_off, const uint8_t *sr, int n_lr,
                            const int64_t *lr_off, const uint8_t *lr, int64_t n_task, const int32_t *t_sr,
                            const int32_t *t_lr, const uint8_t *t_strand, const int32_t *t_qbeg,
                            const int32_t *t_rbeg, const int32_t *t_slen, const int32_t *t_chain, int64_t read_id0,
                            int32_t *nout, int32_t *olist, int32_t *oflag, int32_t *o_qb, int32_t *o_qe,
                            int32_t *o_rb, int32_t *o_re, int32_t *o_score, int32_t *o_truesc, int64_t *stats) {
    const size_t n1 = (size_t)n_task + 1, r1 = (size_t)n_sr + 1;
    std::vector<int64_t> seed_off(r1, 0);
    for (int64_t t = 0; t < n_task; ++t) ++seed_off[(size_t)t_sr[t] + 1];
    for (int i = 0; i < n_sr; ++i) seed_off[(size_t)i + 1] += seed_off[(size_t)i];
    std::vector<int32_t> w(n1), resume(r1), pscore(n1), npk(r1), tlist(n1), cnext(n1);
    std::vector<uint8_t> pass(n1), sel(n1), ext(n1), dec(n1), fdone(r1);
    std::vector<AlnReg> R(n1);
    std::vector<int32_t> ix(n1);
    AlnDev A;
    std::memset(&A, 0, sizeof A);
    A.n_task = n_task;
    A.n_sr = n_sr;
    A.n_lr = n_lr;
    A.read_id0 = read_id0;
    A.seed_off = seed_off.data();
    A.t_sr = t_sr; A.t_lr = t_lr; A.t_qbeg = t_qbeg; A.t_rbeg = t_rbeg; A.t_slen = t_slen; A.t_chain = t_chain;
    A.t_strand = t_strand;
    A.sr_off = sr_off; A.lr_off = lr_off; A.sr = sr; A.lr = lr;
    A.o_qb = o_qb; A.o_qe = o_qe; A.o_rb = o_rb; A.o_re = o_re; A.o_score = o_score; A.o_truesc = o_truesc;
    A.o_w = w.data();
    A.o_pass = pass.data();
    A.sel = sel.data(); A.ext = ext.data(); A.dec = dec.data();
    A.resume = resume.data();
    A.R = R.data(); A.ix = ix.data(); A.pscore = pscore.data(); A.npk = npk.data(); A.fdone = fdone.data();
    A.nout = nout; A.olist = olist; A.oflag = oflag;
    A.tlist = tlist.data(); A.cnext = cnext.data();
    A.a = o->a; A.b = o->b; A.o_del = o->o_del; A.e_del = o->e_del; A.o_ins = o->o_ins; A.e_ins = o->e_ins; A.w = o->w;
    A.max_chain_gap = max_chain_gap;
    A.min_score_per_base = o->min_score_per_base;
    A.drop_ratio = drop_ratio; A.mask_level = mask_level; A.mask_level_redun = mask_level_redun;
    // aln_init_kernel
    for (int64_t t = 0; t < n_task; ++t) alnc::aln_init_task(A, t);
    std::vector<int32_t> hprev((size_t)n1, -1);   // aln_heads_kernel (the device's walk path)
    A.hprev = hprev.data();
    std::vector<AlnBox> box((size_t)n1);   // the walk's packed regions (the device path)
    A.box = box.data();
    for (int r = 0; r < n_sr; ++r) alnc::aln_heads_read(A, r);
    for (int r = 0; r < n_sr; ++r) resume[(size_t)r] = (int32_t)seed_off[(size_t)r];
    int64_t rounds = 0, n_ext = 0, n_patch = 0;
    for (;;) {   // the extension rounds (sw_launch_extend on SEL_EXT tasks, then the walk)
        for (int64_t t = 0; t < n_task; ++t) {
            if (!(sel[(size_t)t] & SEL_EXT)) continue;
            const int s = t_sr[t], l = t_lr[t];
            osw_region g;
            if (osw_extend_seed(o, sr + sr_off[s], (int)(sr_off[s + 1] - sr_off[s]), lr + lr_off[l],
                                (int)(lr_off[l + 1] - lr_off[l]), t_strand[t], t_qbeg[t], t_rbeg[t], t_slen[t], &g))
                return -1;
            o_qb[t] = g.qb; o_qe[t] = g.qe; o_rb[t] = g.rb; o_re[t] = g.re;
            o_score[t] = g.score; o_truesc[t] = g.truesc; w[(size_t)t] = g.w;
            ++n_ext;
        }
        int req = 0;
        for (int r = 0; r < n_sr; ++r) req += alnc::aln_walk_read(A, r, [](int64_t) {});
        ++rounds;
        if (!req) break;
    }
    for (;;) {   // the final pass; patch scores in extra rounds
        std::vector<AlnPatch> reqs;
        for (int r = 0; r < n_sr; ++r) {
            AlnPatch p;
            if (alnc::aln_final_read(A, r, &p)) reqs.push_back(p);
        }
        if (reqs.empty()) break;
        for (const AlnPatch &p : reqs) {
            int qmax = 1;
            for (int i = 0; i < n_sr; ++i) qmax = qmax > (int)(sr_off[i + 1] - sr_off[i]) ? qmax : (int)(sr_off[i + 1] - sr_off[i]);
            const int64_t stride = 2 * ((int64_t)qmax + 2);
            std::vector<int32_t> pool((size_t)stride);
            pscore[(size_t)(seed_off[(size_t)p.read] + p.m)] = alnc::aln_patch_score(A, p, pool.data(), stride);
            npk[(size_t)p.read] = p.m + 1;
            ++n_patch;
        }
    }
    stats[0] = rounds;
    stats[1] = n_ext;
    stats[2] = n_patch;
    return 0;
}
