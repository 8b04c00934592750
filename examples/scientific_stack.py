# numpy / pandas / scipy are preinstalled in every sandbox.
import numpy as np
import pandas as pd
from scipy import stats

rng = np.random.default_rng(7)
df = pd.DataFrame({"a": rng.normal(0.0, 1.0, 500), "b": rng.normal(0.2, 1.0, 500)})
print(df.describe().loc[["mean", "std"]])
t, p = stats.ttest_ind(df["a"], df["b"])
print(f"T-Statistic: {t:.4f}")
print(f"P-Value: {p:.4g}")
