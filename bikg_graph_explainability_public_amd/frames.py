"""Result tables: the reference's `pd.DataFrame({...}).set_index("name").sort_values(by=[key],
ascending=False)` (data.py:651-693, pathways.py:420-429, the latter + `.dropna()`), built once from
numpy arrays instead of through three intermediate frames.  The row order is pandas' own
single-key sort (pandas.core.sorting.nargsort: NaN rows set aside, non-NaN values reversed,
quicksort argsort, reversed back, NaN rows appended in their original order), so ties and NaNs
come out exactly where pandas puts them."""
import numpy as np
import pandas as pd


def name_labels(names):
    """(labels, all_str): the row labels of `names` as an object array and whether pandas infers
    them as strings — what sorted_frame derives from `names` on every call; a caller that builds
    many frames over one unchanging names list computes it once and passes it in."""
    labels = np.fromiter(names, dtype=object, count=len(names))
    return labels, pd.api.types.infer_dtype(labels, skipna=False) == "string"


def sorted_frame(names, columns, key, dropna=False, labels=None):
    """names: row labels (index "name"); columns: {column: 1-D array} in output order; rows
    sorted by `key` descending; dropna drops every row with a NaN in any column.  `labels`:
    name_labels(names), when the caller has it already."""
    cols = {c: np.asarray(v) for c, v in columns.items()}
    s = cols[key]
    nan = np.isnan(s) if s.dtype.kind == "f" else np.zeros(len(s), dtype=bool)
    pos = np.arange(len(s))
    nn, ni = s[~nan][::-1], pos[~nan][::-1]
    order = np.concatenate([ni[nn.argsort(kind="quicksort")][::-1], pos[nan]])
    if dropna:
        bad = np.zeros(len(s), dtype=bool)
        for v in cols.values():
            if v.dtype.kind == "f":
                bad |= np.isnan(v)
        order = order[~bad[order]]
    labels, all_str = name_labels(names) if labels is None else labels
    if all_str:
        # str labels: an object array skips pandas' per-element inference of a list (~0.2 ms at
        # 1.2k names); other label types keep the list constructor (int names -> int64 index)
        index = pd.Index(labels[order], name="name")
    else:
        index = pd.Index(list(names), name="name")[order]
    if len({v.dtype for v in cols.values()}) == 1 and all(v.ndim == 1 for v in cols.values()):
        # one dtype: a single 2-D block (the dict constructor sanitises column by column)
        return pd.DataFrame(np.stack([v[order] for v in cols.values()], axis=1), index=index,
                            columns=list(cols))
    return pd.DataFrame({c: v[order] for c, v in cols.items()}, index=index)
