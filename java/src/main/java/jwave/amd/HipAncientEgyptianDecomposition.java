/*
 * HipAncientEgyptianDecomposition — AncientEgyptianDecomposition
 * (AncientEgyptianDecomposition.java:97-184) over a HipFastWaveletTransform or
 * HipWaveletPacketTransform: an array of any length in ONE native call
 * (jwv_aed_*): the power-of-two pieces (MathToolKit.decompose, largest first)
 * each at full depth, every piece of <= 8192 samples in one varlen launch.
 * Any other wrapped transform, or a wavelet the native path does not cover,
 * runs the reference's Java loop.
 */
package jwave.amd;

import jwave.exceptions.JWaveException;
import jwave.transforms.AncientEgyptianDecomposition;
import jwave.transforms.BasicTransform;

public class HipAncientEgyptianDecomposition extends AncientEgyptianDecomposition {

  private final HipNative.Taps _taps;  // null: the reference's Java loop
  private final int _kind;             // 0 FWT, 1 WPT (JWV_TRANSFORM_*)

  public HipAncientEgyptianDecomposition( BasicTransform basicTransform ) {
    super( basicTransform );
    if( basicTransform instanceof HipFastWaveletTransform ) {
      _taps = ( (HipFastWaveletTransform)basicTransform ).taps( );
      _kind = ( (HipFastWaveletTransform)basicTransform ).kind( );
    } else if( basicTransform instanceof HipWaveletPacketTransform ) {
      _taps = ( (HipWaveletPacketTransform)basicTransform ).taps( );
      _kind = 1;
    } else {
      _taps = null;
      _kind = 0;
    }
  }

  private double[ ] run( boolean fwd, double[ ] a ) throws JWaveException {
    HipNative.Taps t = _taps;
    double[ ] out = new double[ a.length ];
    HipNative.check( HipNative.aed( HipNative.ctx( ), _kind, fwd, a, out, t.L, t.tw, t.scale,
        t.lo, t.hi, t.loR, t.hiR ) );
    return out;
  }

  @Override public double[ ] forward( double[ ] arrTime ) throws JWaveException {
    if( _taps == null )
      return super.forward( arrTime );
    return run( true, arrTime );
  }

  @Override public double[ ] reverse( double[ ] arrHilb ) throws JWaveException {
    if( _taps == null )
      return super.reverse( arrHilb );
    return run( false, arrHilb );
  }
}
