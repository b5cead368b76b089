package server

// Start-command flags and construction of the GPU signature verifier from the
// node configuration (server/config/gpuverify.go).  Patch: in StartCmd
// (server/start.go:20-101) call AddGPUVerifyFlags(cmd) next to the other
// flags; the app constructor (AppCreator) calls NewGPUVerifier with the
// loaded [gpu-verify] section and the app's logger.

import (
	"github.com/spf13/cobra"
	"github.com/spf13/viper"
	"github.com/tendermint/tendermint/libs/log"

	gv "github.com/cosmos/cosmos-sdk/crypto/gpuverify"
	"github.com/cosmos/cosmos-sdk/server/config"
)

// Flag names (viper keys of the [gpu-verify] section).
const (
	FlagGPUVerify         = "gpu-verify.enable"
	FlagGPUVerifyDevices  = "gpu-verify.devices"
	FlagGPUVerifyMaxBatch = "gpu-verify.max-batch"
	FlagGPUVerifyCPUBelow = "gpu-verify.cpu-below"
	FlagGPUVerifyKeyed    = "gpu-verify.keyed"
	FlagGPUVerifyWindow   = "gpu-verify.checktx-window"
)

// AddGPUVerifyFlags registers the flags that override app.toml.
func AddGPUVerifyFlags(cmd *cobra.Command) {
	d := config.DefaultGPUVerifyConfig()
	cmd.Flags().Bool(FlagGPUVerify, d.Enable, "Verify tx signatures on the GPU (libgpuverify)")
	cmd.Flags().String(FlagGPUVerifyDevices, d.Devices, "HIP device ids for signature verification (\"\" = all)")
	cmd.Flags().Int(FlagGPUVerifyMaxBatch, d.MaxBatch, "Largest signature batch per device call")
	cmd.Flags().Int(FlagGPUVerifyCPUBelow, d.CPUBelow, "Signature batches below this size verify on the CPU")
	cmd.Flags().Bool(FlagGPUVerifyKeyed, d.Keyed, "Keep account keys parsed in GPU memory")
	cmd.Flags().Duration(FlagGPUVerifyWindow, d.CheckTxWindow, "Concurrent CheckTx accumulation window")
	for _, f := range []string{FlagGPUVerify, FlagGPUVerifyDevices, FlagGPUVerifyMaxBatch, FlagGPUVerifyCPUBelow,
		FlagGPUVerifyKeyed, FlagGPUVerifyWindow} {
		_ = viper.BindPFlag(f, cmd.Flags().Lookup(f))
	}
}

// NewGPUVerifier opens the verifier the configuration asks for.  Disabled,
// invalid or failing to open (no device, no library): the reference CPU path,
// with the reason logged -- the node runs, never with a changed verdict
// (fail closed, SURVEY.md §5).  The returned closer releases the context.
func NewGPUVerifier(cfg config.GPUVerifyConfig, logger log.Logger) (gv.Verifier, func()) {
	nop := func() {}
	if !cfg.Enable {
		return gv.CPU{}, nop
	}
	if err := cfg.Validate(); err != nil {
		logger.Error("gpu-verify disabled: invalid configuration", "err", err)
		return gv.CPU{}, nop
	}
	ids, _ := cfg.DeviceIDs()
	g, err := gv.Open(ids)
	if err != nil {
		logger.Error("gpu-verify disabled: no device", "err", err)
		return gv.CPU{}, nop
	}
	if err := g.SetOption("max_batch", int64(cfg.MaxBatch)); err != nil {
		logger.Error("gpu-verify: max-batch not applied", "err", err)
	}
	g.CPUBelow, g.Keyed, g.KeyLoadMin = cfg.CPUBelow, cfg.Keyed, cfg.KeyLoadMin
	g.KeyCap, g.EdKeyCap = cfg.KeyCap, cfg.EdKeyCap
	g.Logger = logger.With("module", "gpuverify")
	logger.Info("gpu-verify enabled", "devices", cfg.Devices, "keyed", cfg.Keyed, "cpu-below", cfg.CPUBelow)
	return g, g.Close
}
