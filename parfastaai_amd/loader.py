"""SQLite SCP/tetramer loader (Python mirror of the reference's DB layer).

Same SQL and the same id rules as
  SQLiteHelper        include/pfaai/db_helper.hpp:33-219
  SQLiteSCPDataBase   include/pfaai/scp_db.hpp:59-263
  QTSQLiteSCPDataBase include/pfaai/scp_db.hpp:267-590
so the arrays equal the reference's Lc / F / T (pinned by the fixtures in
tests/golden).  Protein index = order of ``SELECT DISTINCT scp_acc FROM
scp_data``; genome index = ``genome_metadata`` row order; query-DB genome ids
are offset by the number of target genomes.
"""
from __future__ import annotations

import sqlite3

import numpy as np

from .datastruct import NTETRAMERS

SQLITE_OK = 0


class DBError(RuntimeError):
    code = 1  # PFAAI_ERR_SQLITE_DB


def _connect(path):
    try:
        # the reference opens read-write (sqlite3_open); read-only is enough here
        return sqlite3.connect(f"file:{path}?mode=ro", uri=True)
    except sqlite3.Error as e:  # pragma: no cover
        raise DBError(f"Error in opening {path}: {e}") from e


def protein_set(conn, table="scp_data"):
    """dbProteinSet (db_helper.hpp:169-218)."""
    return [r[0] for r in conn.execute(f"SELECT DISTINCT scp_acc FROM {table}")]


def genome_set(conn, table="genome_metadata"):
    """dbGenomeSet (db_helper.hpp:59-107)."""
    return [r[0] for r in conn.execute(f"SELECT genome_name FROM {table}")]


def qt_protein_set(conn):
    """qtDBProteinSet (db_helper.hpp:109-166) on the ATTACHed pair."""
    q = ("SELECT DISTINCT target_table.scp_acc \n"
         "  FROM `main`.scp_data as target_table, `QueryDB`.scp_data as query_table \n"
         "  WHERE target_table.scp_acc = query_table.scp_acc;")
    return [r[0] for r in conn.execute(q)]


def _tetras(conn, prot, schema=None):
    tab = f"{schema}.`{prot}_tetras`" if schema else f"`{prot}_tetras`"
    rows = conn.execute(f"SELECT tetramer, genomes FROM {tab}").fetchall()
    t = np.fromiter((r[0] for r in rows), dtype=np.int64, count=len(rows))
    lens = np.fromiter((len(r[1]) // 4 for r in rows), dtype=np.int64, count=len(rows))
    g = np.frombuffer(b"".join(r[1] for r in rows), dtype="<i4")
    return t, lens, g


def _assemble_f(t_list, p_list, g_list):
    """Order (tetramer, protein, blob order) = scp_db.hpp:167-182's
    ``ORDER BY tetramer, source_table`` over the UNION ALL."""
    t = np.concatenate(t_list) if t_list else np.zeros(0, np.int64)
    p = np.concatenate(p_list) if p_list else np.zeros(0, np.int64)
    g = np.concatenate(g_list) if g_list else np.zeros(0, np.int32)
    order = np.lexsort((p, t))  # stable: keeps blob order inside (t, p)
    F = np.stack([p[order].astype(np.int32), g[order].astype(np.int32)], axis=1)
    Lc = np.bincount(t, minlength=NTETRAMERS).astype(np.int32)
    return Lc, F


def load_db(path):
    """-> dict(protein_set, genome_set, Lc, F, T) for one SCP database."""
    conn = _connect(path)
    try:
        prots = protein_set(conn)
        genomes = genome_set(conn)
        T = np.zeros((len(prots), len(genomes)), dtype=np.int32)
        t_list, p_list, g_list = [], [], []
        for pi, prot in enumerate(prots):
            t, lens, g = _tetras(conn, prot)
            t_list.append(np.repeat(t, lens))
            p_list.append(np.full(len(g), pi, dtype=np.int64))
            g_list.append(g)
            # proteinTetramerCounts (scp_db.hpp:219-262)
            for gid, ln in conn.execute(f"SELECT genome_id, length(tetramers) FROM `{prot}_genomes`"):
                T[pi, gid] = ln // 4
        Lc, F = _assemble_f(t_list, p_list, g_list)
        return dict(protein_set=prots, genome_set=genomes, Lc=Lc, F=F, T=T)
    finally:
        conn.close()


def load_qt(tgt_path, qry_path):
    """-> dict(protein_set, tgt_genome_set, qry_genome_set, Lc, F, T) for
    the query-vs-target pair (QTSQLiteSCPDataBase, scp_db.hpp:267-590)."""
    conn = _connect(tgt_path)
    try:
        conn.execute("ATTACH DATABASE ? as QueryDB", (f"file:{qry_path}?mode=ro",))
    except sqlite3.Error:
        conn.execute("ATTACH DATABASE ? as QueryDB", (qry_path,))
    try:
        prots = qt_protein_set(conn)
        tg = genome_set(conn, "`main`.genome_metadata")
        qg = genome_set(conn, "`QueryDB`.genome_metadata")
        nT = len(tg)
        T = np.zeros((len(prots), nT + len(qg)), dtype=np.int32)
        t_list, p_list, g_list = [], [], []
        for pi, prot in enumerate(prots):
            # inner join on tetramer (scp_db.hpp:459-466): target genomes, then query (+nT)
            q = (f"SELECT target_table.tetramer, target_table.genomes, query_table.genomes "
                 f"FROM main.`{prot}_tetras` as target_table, QueryDB.`{prot}_tetras` as query_table "
                 f"WHERE target_table.tetramer = query_table.tetramer")
            for t, tb, qb in conn.execute(q):
                gt = np.frombuffer(tb, dtype="<i4")
                gq = np.frombuffer(qb, dtype="<i4").astype(np.int64) + nT
                g = np.concatenate([gt.astype(np.int64), gq])
                t_list.append(np.full(len(g), t, dtype=np.int64))
                p_list.append(np.full(len(g), pi, dtype=np.int64))
                g_list.append(g.astype(np.int32))
            # dbProteinTetramerCounts (scp_db.hpp:531-589)
            for gid, ln in conn.execute(f"SELECT genome_id, length(tetramers) FROM main.`{prot}_genomes`"):
                T[pi, gid] += ln // 4
            for gid, ln in conn.execute(f"SELECT genome_id, length(tetramers) FROM QueryDB.`{prot}_genomes`"):
                T[pi, nT + gid] += ln // 4
        Lc, F = _assemble_f(t_list, p_list, g_list)
        return dict(protein_set=prots, tgt_genome_set=tg, qry_genome_set=qg, Lc=Lc, F=F, T=T)
    finally:
        conn.close()
