"""Properties of the generated level programs that the kernels rely on
(host-only: the tables are parsed from the generated headers).

k_set_hash_coop runs the cofactor program through crow::level<..., NOALIAS =
true> (tb_cprog.h), which stores a level's outputs without a barrier after
the output sums: valid only if no output slot of a level is read by another
output's sum of the same level.  Both interpreters also store products
without a barrier after the operand sums: no product slot may be an operand
of the same level."""

import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _tables(header, prefix):
    src = open(os.path.join(ROOT, "teku_amd", "csrc", header)).read()

    def arr(name):
        m = re.search(prefix + name + r"\[\d+\] = \{([^}]*)\}", src)
        return [int(x) for x in m.group(1).split(",")]

    return arr("TYPE_OFF"), arr("TAB")


def _hazards(off, tab):
    out_alias, prod_alias = [], []
    for ty, o in enumerate(off):
        np_, nq, no = tab[o], tab[o + 1], tab[o + 2]
        abeg = o + 3
        bbeg = abeg + np_ + 1
        pout = bbeg + np_ + 1
        qbeg = pout + np_
        obeg = qbeg + nq + 1
        odst = obeg + no + 1
        ent = odst + no

        def terms(b, e):
            return {tab[ent + 2 * i] for i in range(b, e)}

        outs = [tab[odst + k] for k in range(no)]
        for k in range(no):
            rd = terms(tab[qbeg + tab[obeg + k]], tab[qbeg + tab[obeg + k + 1]])
            if any(outs[j] in rd for j in range(no) if j != k):
                out_alias.append(ty)
        reads = set()
        for t in range(np_):
            reads |= terms(tab[abeg + t], tab[abeg + t + 1]) | terms(tab[bbeg + t], tab[bbeg + t + 1])
        if reads & {tab[pout + t] for t in range(np_)}:
            prod_alias.append(ty)
    return out_alias, prod_alias


def test_cofactor_program_has_no_output_or_product_aliasing():
    out_alias, prod_alias = _hazards(*_tables("tb_cofactor_prog.h", "CF_"))
    assert out_alias == [] and prod_alias == []


def test_miller_program_has_no_product_aliasing():
    _, prod_alias = _hazards(*_tables("tb_miller_prog.h", "MP_"))
    assert prod_alias == []
