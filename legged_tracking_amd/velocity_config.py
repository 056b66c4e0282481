"""Config contract of the reference's velocity-tracking env (BASELINE configs[1]).

`make_vel_cfg()` mirrors go1_gym/envs/base/legged_robot_velocity_tracking_config.py:6-421 (the
attributes VelocityTrackingEasyEnv reads), `config_go1_vel` mirrors go1_gym/envs/go1/go1_config.py:8-106
and `train_velocity_config` applies scripts/train_velocity_tracking.py:20-207 (the walk-these-ways
CoRL configuration: 15 commands, gait clock inputs, CoRLRewards, command curriculum), with the
terrain mesh selectable (BASELINE configs[1] runs it on a plane).  Same plain-class machinery as
config.py: `vars(Cfg.x)` returns the attributes in definition order, attributes set later appended.
"""
import math

import numpy as np

from .config import PrefixProto, ParamsProto


def make_vel_cfg():
    """A fresh velocity-tracking Cfg class tree with the reference's defaults."""

    class Cfg(PrefixProto, cli=False):
        class env(PrefixProto, cli=False):
            num_envs = 4096
            num_observations = 235
            num_scalar_observations = 42
            num_privileged_obs = 18
            privileged_future_horizon = 1
            num_actions = 12
            num_observation_history = 15
            env_spacing = 3.
            send_timeouts = True
            episode_length_s = 20
            observe_vel = True
            observe_only_ang_vel = False
            observe_only_lin_vel = False
            observe_yaw = False
            observe_contact_states = False
            observe_command = True
            observe_height_command = False
            observe_gait_commands = False
            observe_timing_parameter = False
            observe_clock_inputs = False
            observe_two_prev_actions = False
            observe_imu = False
            record_video = True
            recording_width_px = 360
            recording_height_px = 240
            recording_mode = "COLOR"
            num_recording_envs = 1
            debug_viz = False
            all_agents_share = False
            priv_observe_friction = True
            priv_observe_friction_indep = True
            priv_observe_ground_friction = False
            priv_observe_ground_friction_per_foot = False
            priv_observe_restitution = True
            priv_observe_base_mass = True
            priv_observe_com_displacement = True
            priv_observe_motor_strength = False
            priv_observe_motor_offset = False
            priv_observe_joint_friction = True
            priv_observe_Kp_factor = True
            priv_observe_Kd_factor = True
            priv_observe_contact_forces = False
            priv_observe_contact_states = False
            priv_observe_body_velocity = False
            priv_observe_foot_height = False
            priv_observe_body_height = False
            priv_observe_gravity = False
            priv_observe_terrain_type = False
            priv_observe_clock_inputs = False
            priv_observe_doubletime_clock_inputs = False
            priv_observe_halftime_clock_inputs = False
            priv_observe_desired_contact_states = False
            priv_observe_dummy_variable = False

        class terrain(PrefixProto, cli=False):
            mesh_type = 'trimesh'
            horizontal_scale = 0.1
            vertical_scale = 0.005
            border_size = 0
            curriculum = True
            static_friction = 1.0
            dynamic_friction = 1.0
            restitution = 0.0
            terrain_noise_magnitude = 0.1
            terrain_smoothness = 0.005
            measure_heights = True
            measured_points_x = [-0.8, -0.7, -0.6, -0.5, -0.4, -0.3, -0.2, -0.1, 0., 0.1, 0.2, 0.3, 0.4, 0.5, 0.6,
                                 0.7, 0.8]
            measured_points_y = [-0.5, -0.4, -0.3, -0.2, -0.1, 0., 0.1, 0.2, 0.3, 0.4, 0.5]
            selected = False
            terrain_kwargs = None
            min_init_terrain_level = 0
            max_init_terrain_level = 5
            terrain_length = 8.
            terrain_width = 8.
            num_rows = 10
            num_cols = 20
            terrain_proportions = [0.1, 0.1, 0.35, 0.25, 0.2]
            slope_treshold = 0.75
            difficulty_scale = 1.
            x_init_range = 1.
            y_init_range = 1.
            yaw_init_range = 0.
            x_init_offset = 0.
            y_init_offset = 0.
            teleport_robots = True
            teleport_thresh = 2.0
            max_platform_height = 0.2
            center_robots = False
            center_span = 5

        class commands(PrefixProto, cli=False):
            command_curriculum = False
            max_reverse_curriculum = 1.
            max_forward_curriculum = 1.
            yaw_command_curriculum = False
            max_yaw_curriculum = 1.
            exclusive_command_sampling = False
            num_commands = 3
            resampling_time = 10.
            subsample_gait = False
            gait_interval_s = 10.
            vel_interval_s = 10.
            jump_interval_s = 20.
            jump_duration_s = 0.1
            jump_height = 0.3
            heading_command = True
            global_reference = False
            observe_accel = False
            distributional_commands = False
            curriculum_type = "RewardThresholdCurriculum"
            lipschitz_threshold = 0.9
            num_lin_vel_bins = 20
            lin_vel_step = 0.3
            num_ang_vel_bins = 20
            ang_vel_step = 0.3
            distribution_update_extension_distance = 1
            curriculum_seed = 100
            lin_vel_x = [-1.0, 1.0]
            lin_vel_y = [-1.0, 1.0]
            ang_vel_yaw = [-1, 1]
            body_height_cmd = [-0.05, 0.05]
            impulse_height_commands = False
            limit_vel_x = [-10.0, 10.0]
            limit_vel_y = [-0.6, 0.6]
            limit_vel_yaw = [-10.0, 10.0]
            limit_body_height = [-0.05, 0.05]
            limit_gait_phase = [0, 0.01]
            limit_gait_offset = [0, 0.01]
            limit_gait_bound = [0, 0.01]
            limit_gait_frequency = [2.0, 2.01]
            limit_gait_duration = [0.49, 0.5]
            limit_footswing_height = [0.06, 0.061]
            limit_body_pitch = [0.0, 0.01]
            limit_body_roll = [0.0, 0.01]
            limit_aux_reward_coef = [0.0, 0.01]
            limit_compliance = [0.0, 0.01]
            limit_stance_width = [0.0, 0.01]
            limit_stance_length = [0.0, 0.01]
            num_bins_vel_x = 25
            num_bins_vel_y = 3
            num_bins_vel_yaw = 25
            num_bins_body_height = 1
            num_bins_gait_frequency = 11
            num_bins_gait_phase = 11
            num_bins_gait_offset = 2
            num_bins_gait_bound = 2
            num_bins_gait_duration = 3
            num_bins_footswing_height = 1
            num_bins_body_pitch = 1
            num_bins_body_roll = 1
            num_bins_aux_reward_coef = 1
            num_bins_compliance = 1
            num_bins_stance_width = 1
            num_bins_stance_length = 1
            heading = [-3.14, 3.14]
            gait_phase_cmd_range = [0.0, 0.01]
            gait_offset_cmd_range = [0.0, 0.01]
            gait_bound_cmd_range = [0.0, 0.01]
            gait_frequency_cmd_range = [2.0, 2.01]
            gait_duration_cmd_range = [0.49, 0.5]
            footswing_height_range = [0.06, 0.061]
            body_pitch_range = [0.0, 0.01]
            body_roll_range = [0.0, 0.01]
            aux_reward_coef_range = [0.0, 0.01]
            compliance_range = [0.0, 0.01]
            stance_width_range = [0.0, 0.01]
            stance_length_range = [0.0, 0.01]
            exclusive_phase_offset = True
            binary_phases = False
            pacing_offset = False
            balance_gait_distribution = True
            gaitwise_curricula = True

        class curriculum_thresholds(PrefixProto, cli=False):
            tracking_lin_vel = 0.8
            tracking_ang_vel = 0.5
            tracking_contacts_shaped_force = 0.8
            tracking_contacts_shaped_vel = 0.8

        class init_state(PrefixProto, cli=False):
            pos = [0.0, 0.0, 1.]
            rot = [0.0, 0.0, 0.0, 1.0]
            lin_vel = [0.0, 0.0, 0.0]
            ang_vel = [0.0, 0.0, 0.0]
            default_joint_angles = {"joint_a": 0., "joint_b": 0.}

        class control(PrefixProto, cli=False):
            control_type = 'actuator_net'
            stiffness = {'joint_a': 10.0, 'joint_b': 15.}
            damping = {'joint_a': 1.0, 'joint_b': 1.5}
            action_scale = 0.5
            hip_scale_reduction = 1.0
            decimation = 4

        class asset(PrefixProto, cli=False):
            file = ""
            foot_name = "None"
            penalize_contacts_on = []
            terminate_after_contacts_on = []
            disable_gravity = False
            collapse_fixed_joints = True
            fix_base_link = False
            default_dof_drive_mode = 3
            self_collisions = 0
            replace_cylinder_with_capsule = True
            flip_visual_attachments = True
            density = 0.001
            angular_damping = 0.
            linear_damping = 0.
            max_angular_velocity = 1000.
            max_linear_velocity = 1000.
            armature = 0.
            thickness = 0.01

        class domain_rand(PrefixProto, cli=False):
            rand_interval_s = 10
            randomize_rigids_after_start = True
            randomize_friction = True
            friction_range = [0.5, 1.25]
            randomize_restitution = False
            restitution_range = [0, 1.0]
            randomize_base_mass = False
            added_mass_range = [-1., 1.]
            randomize_com_displacement = False
            com_displacement_range = [-0.15, 0.15]
            randomize_motor_strength = False
            motor_strength_range = [0.9, 1.1]
            randomize_Kp_factor = False
            Kp_factor_range = [0.8, 1.3]
            randomize_Kd_factor = False
            Kd_factor_range = [0.5, 1.5]
            gravity_rand_interval_s = 7
            gravity_impulse_duration = 1.0
            randomize_gravity = False
            gravity_range = [-1.0, 1.0]
            push_robots = True
            push_interval_s = 15
            max_push_vel_xy = 1.
            randomize_lag_timesteps = True
            lag_timesteps = 6

        class rewards(PrefixProto, cli=False):
            only_positive_rewards = True
            only_positive_rewards_ji22_style = False
            sigma_rew_neg = 5
            reward_container_name = "CoRLRewards"
            tracking_sigma = 0.25
            tracking_sigma_lat = 0.25
            tracking_sigma_long = 0.25
            tracking_sigma_yaw = 0.25
            soft_dof_pos_limit = 1.
            soft_dof_vel_limit = 1.
            soft_torque_limit = 1.
            base_height_target = 1.
            max_contact_force = 100.
            use_terminal_body_height = False
            terminal_body_height = 0.20
            use_terminal_foot_height = False
            terminal_foot_height = -0.005
            use_terminal_roll_pitch = False
            terminal_body_ori = 0.5
            kappa_gait_probs = 0.07
            gait_force_sigma = 50.
            gait_vel_sigma = 0.5
            footswing_height = 0.09

        class reward_scales(ParamsProto, cli=False):
            termination = -0.0
            tracking_lin_vel = 1.0
            tracking_ang_vel = 0.5
            lin_vel_z = -2.0
            ang_vel_xy = -0.05
            orientation = -0.
            torques = -0.00001
            dof_vel = -0.
            dof_acc = -2.5e-7
            base_height = -0.
            feet_air_time = 1.0
            collision = -1.
            feet_stumble = -0.0
            action_rate = -0.01
            stand_still = -0.
            tracking_lin_vel_lat = 0.
            tracking_lin_vel_long = 0.
            tracking_contacts = 0.
            tracking_contacts_shaped = 0.
            tracking_contacts_shaped_force = 0.
            tracking_contacts_shaped_vel = 0.
            jump = 0.0
            energy = 0.0
            energy_expenditure = 0.0
            survival = 0.0
            dof_pos_limits = 0.0
            feet_contact_forces = 0.
            feet_slip = 0.
            feet_clearance_cmd_linear = 0.
            dof_pos = 0.
            action_smoothness_1 = 0.
            action_smoothness_2 = 0.
            base_motion = 0.
            feet_impact_vel = 0.0
            raibert_heuristic = 0.0

        class normalization(PrefixProto, cli=False):
            clip_observations = 100.
            clip_actions = 100.
            friction_range = [0.05, 4.5]
            ground_friction_range = [0.05, 4.5]
            restitution_range = [0, 1.0]
            added_mass_range = [-1., 3.]
            com_displacement_range = [-0.1, 0.1]
            motor_strength_range = [0.9, 1.1]
            motor_offset_range = [-0.05, 0.05]
            Kp_factor_range = [0.8, 1.3]
            Kd_factor_range = [0.5, 1.5]
            joint_friction_range = [0.0, 0.7]
            contact_force_range = [0.0, 50.0]
            contact_state_range = [0.0, 1.0]
            body_velocity_range = [-6.0, 6.0]
            foot_height_range = [0.0, 0.15]
            body_height_range = [0.0, 0.60]
            gravity_range = [-1.0, 1.0]
            motion = [-0.01, 0.01]

        class obs_scales(PrefixProto, cli=False):
            lin_vel = 2.0
            ang_vel = 0.25
            dof_pos = 1.0
            dof_vel = 0.05
            imu = 0.1
            height_measurements = 5.0
            friction_measurements = 1.0
            body_height_cmd = 2.0
            gait_phase_cmd = 1.0
            gait_freq_cmd = 1.0
            footswing_height_cmd = 0.15
            body_pitch_cmd = 0.3
            body_roll_cmd = 0.3
            aux_reward_cmd = 1.0
            compliance_cmd = 1.0
            stance_width_cmd = 1.0
            stance_length_cmd = 1.0
            segmentation_image = 1.0
            rgb_image = 1.0
            depth_image = 1.0

        class noise(PrefixProto, cli=False):
            add_noise = True
            noise_level = 1.0

        class noise_scales(PrefixProto, cli=False):
            dof_pos = 0.01
            dof_vel = 1.5
            lin_vel = 0.1
            ang_vel = 0.2
            imu = 0.1
            gravity = 0.05
            contact_states = 0.05
            height_measurements = 0.1
            friction_measurements = 0.0
            segmentation_image = 0.0
            rgb_image = 0.0
            depth_image = 0.0

        class viewer(PrefixProto, cli=False):
            ref_env = 0
            pos = [10, 0, 6]
            lookat = [11., 5, 3.]

        class sim(PrefixProto, cli=False):
            dt = 0.005
            substeps = 1
            gravity = [0., 0., -9.81]
            up_axis = 1
            use_gpu_pipeline = True

            class physx(PrefixProto, cli=False):
                num_threads = 10
                solver_type = 1
                num_position_iterations = 4
                num_velocity_iterations = 0
                contact_offset = 0.01
                rest_offset = 0.0
                bounce_threshold_velocity = 0.5
                max_depenetration_velocity = 1.0
                max_gpu_contact_pairs = 2 ** 23
                default_buffer_size_multiplier = 5
                contact_collection = 2

    return Cfg


def config_go1_vel(C):
    """go1_gym/envs/go1/go1_config.py:8-106."""
    _ = C.init_state
    _.pos = [0.0, 0.0, 0.34]
    _.default_joint_angles = {'FL_hip_joint': 0.1, 'RL_hip_joint': 0.1, 'FR_hip_joint': -0.1, 'RR_hip_joint': -0.1,
                              'FL_thigh_joint': 0.8, 'RL_thigh_joint': 1., 'FR_thigh_joint': 0.8,
                              'RR_thigh_joint': 1., 'FL_calf_joint': -1.5, 'RL_calf_joint': -1.5,
                              'FR_calf_joint': -1.5, 'RR_calf_joint': -1.5}
    _ = C.control
    _.control_type = 'P'
    _.stiffness = {'joint': 20.}
    _.damping = {'joint': 0.5}
    _.action_scale = 0.25
    _.hip_scale_reduction = 0.5
    _.decimation = 4
    _ = C.asset
    _.file = '{MINI_GYM_ROOT_DIR}/resources/robots/go1/urdf/go1.urdf'
    _.foot_name = "foot"
    _.penalize_contacts_on = ["thigh", "calf"]
    _.terminate_after_contacts_on = ["base"]
    _.self_collisions = 0
    _.flip_visual_attachments = False
    _.fix_base_link = False
    _ = C.rewards
    _.soft_dof_pos_limit = 0.9
    _.base_height_target = 0.34
    _ = C.reward_scales
    _.torques = -0.0001
    _.action_rate = -0.01
    _.dof_pos_limits = -10.0
    _.orientation = -5.
    _.base_height = -30.
    _ = C.terrain
    _.mesh_type = 'trimesh'
    _.measure_heights = False
    _.terrain_noise_magnitude = 0.0
    _.teleport_robots = True
    _.border_size = 50
    _.terrain_proportions = [0, 0, 0, 0, 0, 0, 0, 0, 1.0]
    _.curriculum = False
    _ = C.env
    _.num_observations = 42
    _.observe_vel = False
    _.num_envs = 4000
    _ = C.commands
    _.lin_vel_x = [-1.0, 1.0]
    _.lin_vel_y = [-1.0, 1.0]
    _ = C.commands
    _.heading_command = False
    _.resampling_time = 10.0
    _.command_curriculum = True
    _.num_lin_vel_bins = 30
    _.num_ang_vel_bins = 30
    _.lin_vel_x = [-0.6, 0.6]
    _.lin_vel_y = [-0.6, 0.6]
    _.ang_vel_yaw = [-1, 1]
    _ = C.domain_rand
    _.randomize_base_mass = True
    _.added_mass_range = [-1, 3]
    _.push_robots = False
    _.max_push_vel_xy = 0.5
    _.randomize_friction = True
    _.friction_range = [0.05, 4.5]
    _.randomize_restitution = True
    _.restitution_range = [0.0, 1.0]
    _.restitution = 0.5
    _.randomize_com_displacement = True
    _.com_displacement_range = [-0.1, 0.1]
    _.randomize_motor_strength = True
    _.motor_strength_range = [0.9, 1.1]
    _.randomize_Kp_factor = False
    _.Kp_factor_range = [0.8, 1.3]
    _.randomize_Kd_factor = False
    _.Kd_factor_range = [0.5, 1.5]
    _.rand_interval_s = 6


def apply_train_velocity_tracking(C):
    """scripts/train_velocity_tracking.py:20-207 (the Cfg edits before VelocityTrackingEasyEnv)."""
    config_go1_vel(C)
    c = C.commands
    c.num_lin_vel_bins = 30
    c.num_ang_vel_bins = 30
    t = C.curriculum_thresholds
    t.tracking_ang_vel = 0.7
    t.tracking_lin_vel = 0.8
    t.tracking_contacts_shaped_vel = 0.90
    t.tracking_contacts_shaped_force = 0.90
    c.distributional_commands = True
    d, e, r, rs = C.domain_rand, C.env, C.rewards, C.reward_scales
    d.lag_timesteps = 6
    d.randomize_lag_timesteps = True
    C.control.control_type = "actuator_net"
    d.randomize_rigids_after_start = False
    e.priv_observe_motion = False
    e.priv_observe_gravity_transformed_motion = False
    d.randomize_friction_indep = False
    e.priv_observe_friction_indep = False
    d.randomize_friction = True
    e.priv_observe_friction = True
    d.friction_range = [0.1, 3.0]
    d.randomize_restitution = True
    e.priv_observe_restitution = True
    d.restitution_range = [0.0, 0.4]
    d.randomize_base_mass = True
    e.priv_observe_base_mass = False
    d.added_mass_range = [-1.0, 3.0]
    d.randomize_gravity = True
    d.gravity_range = [-1.0, 1.0]
    d.gravity_rand_interval_s = 8.0
    d.gravity_impulse_duration = 0.99
    e.priv_observe_gravity = False
    d.randomize_com_displacement = False
    d.com_displacement_range = [-0.15, 0.15]
    e.priv_observe_com_displacement = False
    d.randomize_ground_friction = True
    e.priv_observe_ground_friction = False
    e.priv_observe_ground_friction_per_foot = False
    d.ground_friction_range = [0.0, 0.0]
    d.randomize_motor_strength = True
    d.motor_strength_range = [0.9, 1.1]
    e.priv_observe_motor_strength = False
    d.randomize_motor_offset = True
    d.motor_offset_range = [-0.02, 0.02]
    e.priv_observe_motor_offset = False
    d.push_robots = False
    d.randomize_Kp_factor = False
    e.priv_observe_Kp_factor = False
    d.randomize_Kd_factor = False
    e.priv_observe_Kd_factor = False
    e.priv_observe_body_velocity = False
    e.priv_observe_body_height = False
    e.priv_observe_desired_contact_states = False
    e.priv_observe_contact_forces = False
    e.priv_observe_foot_displacement = False
    e.priv_observe_gravity_transformed_foot_displacement = False
    e.num_privileged_obs = 2
    e.num_observation_history = 30
    rs.feet_contact_forces = 0.0
    d.rand_interval_s = 4
    c.num_commands = 15
    e.observe_two_prev_actions = True
    e.observe_yaw = False
    e.num_observations = 70
    e.num_scalar_observations = 70
    e.observe_gait_commands = True
    e.observe_timing_parameter = False
    e.observe_clock_inputs = True
    d.tile_height_range = [-0.0, 0.0]
    d.tile_height_curriculum = False
    d.tile_height_update_interval = 1000000
    d.tile_height_curriculum_step = 0.01
    tr = C.terrain
    tr.border_size = 0.0
    tr.mesh_type = "trimesh"
    tr.num_cols = 30
    tr.num_rows = 30
    tr.terrain_width = 5.0
    tr.terrain_length = 5.0
    tr.x_init_range = 0.2
    tr.y_init_range = 0.2
    tr.teleport_thresh = 0.3
    tr.teleport_robots = False
    tr.center_robots = True
    tr.center_span = 4
    tr.horizontal_scale = 0.10
    tr.terrain_proportions = [0.99] * 10
    r.use_terminal_foot_height = False
    r.use_terminal_body_height = True
    r.terminal_body_height = 0.05
    r.use_terminal_roll_pitch = True
    r.terminal_body_ori = 1.6
    c.resampling_time = 10
    rs.feet_slip = -0.04
    rs.action_smoothness_1 = -0.1
    rs.action_smoothness_2 = -0.1
    rs.dof_vel = -1e-4
    rs.dof_pos = -0.0
    rs.jump = 10.0
    rs.base_height = 0.0
    r.base_height_target = 0.30
    rs.estimation_bonus = 0.0
    rs.raibert_heuristic = -10.0
    rs.feet_impact_vel = -0.0
    rs.feet_clearance = -0.0
    rs.feet_clearance_cmd = -0.0
    rs.feet_clearance_cmd_linear = -30.0
    rs.orientation = 0.0
    rs.orientation_control = -5.0
    rs.tracking_stance_width = -0.0
    rs.tracking_stance_length = -0.0
    rs.lin_vel_z = -0.02
    rs.ang_vel_xy = -0.001
    rs.feet_air_time = 0.0
    rs.hop_symmetry = 0.0
    r.kappa_gait_probs = 0.07
    r.gait_force_sigma = 100.
    r.gait_vel_sigma = 10.
    rs.tracking_contacts_shaped_force = 4.0
    rs.tracking_contacts_shaped_vel = 4.0
    rs.collision = -5.0
    r.reward_container_name = "CoRLRewards"
    r.only_positive_rewards = False
    r.only_positive_rewards_ji22_style = True
    r.sigma_rew_neg = 0.02
    c.lin_vel_x = [-1.0, 1.0]
    c.lin_vel_y = [-0.6, 0.6]
    c.ang_vel_yaw = [-1.0, 1.0]
    c.body_height_cmd = [-0.25, 0.15]
    c.gait_frequency_cmd_range = [2.0, 4.0]
    c.gait_phase_cmd_range = [0.0, 1.0]
    c.gait_offset_cmd_range = [0.0, 1.0]
    c.gait_bound_cmd_range = [0.0, 1.0]
    c.gait_duration_cmd_range = [0.5, 0.5]
    c.footswing_height_range = [0.03, 0.35]
    c.body_pitch_range = [-0.4, 0.4]
    c.body_roll_range = [-0.0, 0.0]
    c.stance_width_range = [0.10, 0.45]
    c.stance_length_range = [0.35, 0.45]
    c.limit_vel_x = [-5.0, 5.0]
    c.limit_vel_y = [-0.6, 0.6]
    c.limit_vel_yaw = [-5.0, 5.0]
    c.limit_body_height = [-0.25, 0.15]
    c.limit_gait_frequency = [2.0, 4.0]
    c.limit_gait_phase = [0.0, 1.0]
    c.limit_gait_offset = [0.0, 1.0]
    c.limit_gait_bound = [0.0, 1.0]
    c.limit_gait_duration = [0.5, 0.5]
    c.limit_footswing_height = [0.03, 0.35]
    c.limit_body_pitch = [-0.4, 0.4]
    c.limit_body_roll = [-0.0, 0.0]
    c.limit_stance_width = [0.10, 0.45]
    c.limit_stance_length = [0.35, 0.45]
    c.num_bins_vel_x = 21
    c.num_bins_vel_y = 1
    c.num_bins_vel_yaw = 21
    c.num_bins_body_height = 1
    c.num_bins_gait_frequency = 1
    c.num_bins_gait_phase = 1
    c.num_bins_gait_offset = 1
    c.num_bins_gait_bound = 1
    c.num_bins_gait_duration = 1
    c.num_bins_footswing_height = 1
    c.num_bins_body_roll = 1
    c.num_bins_body_pitch = 1
    c.num_bins_stance_width = 1
    n = C.normalization
    n.friction_range = [0, 1]
    n.ground_friction_range = [0, 1]
    tr.yaw_init_range = 3.14
    n.clip_actions = 10.0
    c.exclusive_phase_offset = False
    c.pacing_offset = False
    c.binary_phases = True
    c.gaitwise_curricula = True


def train_velocity_config(n_envs=4096, mesh_type="plane"):
    """The Cfg scripts/train_velocity_tracking.py builds, with num_envs and the terrain mesh set
    (BASELINE configs[1]: 4096 envs on a plane)."""
    C = make_vel_cfg()
    apply_train_velocity_tracking(C)
    C.env.num_envs = n_envs
    C.terrain.mesh_type = mesh_type
    return C


# ------------------------------------------------------------------ derived values
def vel_derived(cfg):
    """LeggedRobot._parse_cfg (legged_robot_velocity_tracking.py:1734-1750) and the interval math of
    _post_physics_step_callback / _resample_commands (:702, :715, :732-733)."""
    dt = cfg.control.decimation * cfg.sim.dt
    d = dict(dt=dt, max_episode_length=float(np.ceil(cfg.env.episode_length_s / dt)))
    d["rand_interval"] = int(np.ceil(cfg.domain_rand.rand_interval_s / dt))
    d["gravity_rand_interval"] = int(np.ceil(cfg.domain_rand.gravity_rand_interval_s / dt))
    d["gravity_rand_duration"] = int(np.ceil(d["gravity_rand_interval"] * cfg.domain_rand.gravity_impulse_duration))
    d["resample_interval"] = int(cfg.commands.resampling_time / dt)
    d["curriculum_ep_len"] = min(d["max_episode_length"], d["resample_interval"])
    scales = {}
    for k, v in vars(cfg.reward_scales).items():
        if v != 0:
            scales[k] = v * dt
    d["reward_scales"] = scales
    return d


CATEGORIES = ("pronk", "trot", "pace", "bound")  # gaitwise_curricula (:1319-1321)
CURRICULUM_KEYS = ("x_vel", "y_vel", "yaw_vel", "body_height", "gait_frequency", "gait_phase", "gait_offset",
                   "gait_bounds", "gait_duration", "footswing_height", "body_pitch", "body_roll", "stance_width",
                   "stance_length", "aux_reward_coef")
# _resample_commands (:756-757): the neighbourhood a successful bin spreads to, per curriculum key
LOCAL_RANGE = (0.55, 0.55, 0.55, 0.55, 0.35, 0.25, 0.25, 0.25, 0.25, 1.0, 1.0, 1.0, 1.0, 1.0, 1.0)
TASK_KEYS = ("tracking_lin_vel", "tracking_ang_vel", "tracking_contacts_shaped_force", "tracking_contacts_shaped_vel")


def curriculum_key_ranges(cfg):
    """(low, high, n_bins) per curriculum key (_init_command_distribution :1328-1374)."""
    c = cfg.commands
    lim = [c.limit_vel_x, c.limit_vel_y, c.limit_vel_yaw, c.limit_body_height, c.limit_gait_frequency,
           c.limit_gait_phase, c.limit_gait_offset, c.limit_gait_bound, c.limit_gait_duration,
           c.limit_footswing_height, c.limit_body_pitch, c.limit_body_roll, c.limit_stance_width,
           c.limit_stance_length, c.limit_aux_reward_coef]
    nb = [c.num_bins_vel_x, c.num_bins_vel_y, c.num_bins_vel_yaw, c.num_bins_body_height, c.num_bins_gait_frequency,
          c.num_bins_gait_phase, c.num_bins_gait_offset, c.num_bins_gait_bound, c.num_bins_gait_duration,
          c.num_bins_footswing_height, c.num_bins_body_pitch, c.num_bins_body_roll, c.num_bins_stance_width,
          c.num_bins_stance_length, c.num_bins_aux_reward_coef]
    return [(float(l[0]), float(l[1]), int(b)) for l, b in zip(lim, nb)]


def curriculum_grid(cfg):
    """Curriculum.__init__ (curriculum.py:28-55): the (15, n_bins) f64 grid of bin centroids, the
    per-key bin sizes, and the initial weights of set_to(low, high) (:18-26, velocity :1382-1401)."""
    kr = curriculum_key_ranges(cfg)
    axes = []
    for lo, hi, nbin in kr:
        bs = (hi - lo) / nbin
        axes.append(np.linspace(lo + bs / 2, hi - bs / 2, nbin))
    raw = np.stack(np.meshgrid(*axes, indexing='ij'))
    grid = raw.reshape([len(kr), -1])
    bin_sizes = np.array([(hi - lo) / nbin for lo, hi, nbin in kr])
    c = cfg.commands
    low = np.array([c.lin_vel_x[0], c.lin_vel_y[0], c.ang_vel_yaw[0], c.body_height_cmd[0],
                    c.gait_frequency_cmd_range[0], c.gait_phase_cmd_range[0], c.gait_offset_cmd_range[0],
                    c.gait_bound_cmd_range[0], c.gait_duration_cmd_range[0], c.footswing_height_range[0],
                    c.body_pitch_range[0], c.body_roll_range[0], c.stance_width_range[0],
                    c.stance_length_range[0], c.aux_reward_coef_range[0]])
    high = np.array([c.lin_vel_x[1], c.lin_vel_y[1], c.ang_vel_yaw[1], c.body_height_cmd[1],
                     c.gait_frequency_cmd_range[1], c.gait_phase_cmd_range[1], c.gait_offset_cmd_range[1],
                     c.gait_bound_cmd_range[1], c.gait_duration_cmd_range[1], c.footswing_height_range[1],
                     c.body_pitch_range[1], c.body_roll_range[1], c.stance_width_range[1],
                     c.stance_length_range[1], c.aux_reward_coef_range[1]])
    inds = np.logical_and(grid >= low[:, None], grid <= high[:, None]).all(axis=0)
    w = np.zeros(grid.shape[1])
    w[inds] = 1.0
    return grid, bin_sizes, w


def commands_scale(cfg):
    """_init_buffers (:1214-1221): per-command observation scales, f32."""
    s = cfg.obs_scales
    v = [s.lin_vel, s.lin_vel, s.ang_vel, s.body_height_cmd, s.gait_freq_cmd, s.gait_phase_cmd, s.gait_phase_cmd,
         s.gait_phase_cmd, s.gait_phase_cmd, s.footswing_height_cmd, s.body_pitch_cmd, s.body_roll_cmd,
         s.stance_width_cmd, s.stance_length_cmd, s.aux_reward_cmd]
    return np.asarray(v[:cfg.commands.num_commands], np.float32)


def get_scale_shift(r):
    """go1_gym/utils/math_utils.py:35-38."""
    return 2. / (r[1] - r[0]), (r[1] + r[0]) / 2.


del math
