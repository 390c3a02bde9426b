"""eao_replay_profile slots (replay.cpp prof[]): times in us, counts marked #."""
NAMES = {0: "frame", 1: "local_mapping", 2: "#forest_launch", 3: "forest_complete", 4: "#np_launch",
         5: "np_relaunch", 6: "#frame_start", 7: "frame_start_rt", 8: "#frames", 9: "#spec_np", 10: "#lm_forests", 11: "lm_forest",
         12: "steps1-3", 13: "steps4-9", 14: "frame_start_total", 15: "assoc_loop", 16: "same_cls_flush",
         17: "pending_flush", 18: "kick", 19: "launch", 20: "#retire", 21: "retire", 22: "kick_scan",
         23: "pack", 24: "lm_flush", 25: "lm_stats", 26: "lm_merge_overlap", 27: "#ms_skip", 28: "update", 29: "lm_overlap", 30: "frame_end", 31: "#bts_scan",
         32: "ms_pass12", 33: "ms_pose", 34: "ms_pass3", 35: "ms_corners", 36: "#ms_pts", 37: "big_to_small", 38: "bts_filter",
         39: "forest_spin", 40: "forest_erase", 41: "fs_spin", 42: "spin_fs", 43: "spin_loop", 44: "spin_end", 45: "spin_lm", 46: "spin_steps1-9", 47: "spin_samecls", 48: "spin_np", 49: "spin_pro", 50: "spin_t", 51: "spin_update", 52: "lookahead", 53: "#lookahead", 54: "fs_pack", 55: "#fs_pack_pts",
         56: "fs_prep_finish", 57: "fs_kick", 58: "begin_to_fs_launch", 59: "#fs_launch"}
