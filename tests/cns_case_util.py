"""Turn golden consensus cases (tests/golden/casefmt.py) into GPU-path inputs."""
from proovread_amd import cns


def case_inputs(case):
    noref = case.p("noref") == "1"
    if noref:
        lr = cns.LongRead(case.ref_id, None, None, "", len(case.ref[1]))
    else:
        lr = cns.LongRead(case.ref_id, case.ref[1], case.ref[3], case.ref_desc)
    alns = [cns.SamRecord.from_line(l) for l in case.sam]
    params = cns.CnsParams(
        coverage=float(case.p("coverage")),
        max_ins_length=int(case.p("max_ins_length")),
        use_ref_qual=(case.p("use_ref_qual") == "1") and not noref,
        qual_weighted=case.p("qual_weighted") == "1",
        detect_chimera=case.p("detect_chimera") == "1",
    )
    return lr, alns, params


def params_key(p):
    return (p.coverage, p.max_ins_length, p.use_ref_qual, p.qual_weighted, p.detect_chimera)
