"""summary.csv writer/reader (utils/storage_utils.py:36-84 of the reference): one
header row of the stats-dict keys, then one row per epoch."""
import csv
import os


def save_statistics(experiment_log_dir, filename, stats_dict, current_epoch, continue_from_mode=False,
                    save_full_dict=False):
    path = os.path.join(experiment_log_dir, filename)
    with open(path, "a" if continue_from_mode else "w") as f:
        writer = csv.writer(f)
        if not continue_from_mode:
            writer.writerow(list(stats_dict.keys()))
        if save_full_dict:
            for idx in range(len(list(stats_dict.values())[0])):
                writer.writerow([v[idx] for v in stats_dict.values()])
        else:
            writer.writerow([v[current_epoch] for v in stats_dict.values()])
    return path


def load_statistics(experiment_log_dir, filename):
    with open(os.path.join(experiment_log_dir, filename)) as f:
        lines = f.readlines()
    keys = lines[0].split(",")
    stats = {k: [] for k in keys}
    for line in lines[1:]:
        for idx, value in enumerate(line.split(",")):
            stats[keys[idx]].append(value)
    return stats
