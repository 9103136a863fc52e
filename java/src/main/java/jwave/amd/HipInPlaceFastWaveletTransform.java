/*
 * HipInPlaceFastWaveletTransform — InPlaceFastWaveletTransform
 * (InPlaceFastWaveletTransform.java:70-120) on libjwave_hip.so.  The in-place
 * calls overwrite the caller's array with the result and return that same
 * reference, as the reference does; each is ONE native call whose input and
 * output are the caller's array (the shim stages the input before the call
 * and writes the array only after a successful one, so a failing call leaves
 * it untouched, like the reference's arraycopy after super.forward).  The
 * inherited out-of-place forward/reverse(double[], int) run natively too.
 * Wavelets the native path does not reproduce fall back to the Java code.
 */
package jwave.amd;

import jwave.exceptions.JWaveException;
import jwave.exceptions.JWaveFailure;
import jwave.transforms.InPlaceFastWaveletTransform;
import jwave.transforms.wavelets.Wavelet;

public class HipInPlaceFastWaveletTransform extends InPlaceFastWaveletTransform
    implements HipTransform {

  private final HipNative.Taps _taps;

  public HipInPlaceFastWaveletTransform( Wavelet wavelet ) {
    super( wavelet );
    _taps = HipNative.tapsFor( wavelet );
  }

  @Override public HipNative.Taps taps( ) { return _taps; }

  @Override public int kind( ) { return 0; }

  @Override public double[ ] forward( double[ ] arrTime, int level ) throws JWaveException {
    if( _taps == null )
      return super.forward( arrTime, level );
    double[ ] out = new double[ arrTime.length ];
    HipNative.check( HipNative.t1( 0, true, arrTime, out, level, _taps ) );
    return out;
  }

  @Override public double[ ] reverse( double[ ] arrHilb, int level ) throws JWaveException {
    if( _taps == null )
      return super.reverse( arrHilb, level );
    double[ ] out = new double[ arrHilb.length ];
    HipNative.check( HipNative.t1( 0, false, arrHilb, out, level, _taps ) );
    return out;
  }

  // forwardInPlace(a) = super.forward(a) (WaveletTransform.java:77-88: the
  // power-of-two check with its message, then the maximal level) + arraycopy
  @Override public double[ ] forwardInPlace( double[ ] arrTime ) throws JWaveException {
    if( _taps == null )
      return super.forwardInPlace( arrTime );
    if( !isBinary( arrTime.length ) )
      throw new JWaveFailure( "WaveletTransform#forward - "
          + "given array length is not 2^p | p E N ... = 1, 2, 4, 8, 16, 32, .. "
          + "please use the Ancient Egyptian Decomposition for any other array length!" );
    return forwardInPlace( arrTime, calcExponent( arrTime.length ) );
  }

  @Override public double[ ] forwardInPlace( double[ ] arrTime, int level ) throws JWaveException {
    if( _taps == null )
      return super.forwardInPlace( arrTime, level );
    HipNative.check( HipNative.t1( 0, true, arrTime, arrTime, level, _taps ) );
    return arrTime;
  }

  @Override public double[ ] reverseInPlace( double[ ] arrHilb ) throws JWaveException {
    if( _taps == null )
      return super.reverseInPlace( arrHilb );
    if( !isBinary( arrHilb.length ) )
      throw new JWaveFailure( "WaveletTransform#reverse - "
          + "given array length is not 2^p | p E N ... = 1, 2, 4, 8, 16, 32, .. "
          + "please use the Ancient Egyptian Decomposition for any other array length!" );
    return reverseInPlace( arrHilb, calcExponent( arrHilb.length ) );
  }

  @Override public double[ ] reverseInPlace( double[ ] arrHilb, int level ) throws JWaveException {
    if( _taps == null )
      return super.reverseInPlace( arrHilb, level );
    HipNative.check( HipNative.t1( 0, false, arrHilb, arrHilb, level, _taps ) );
    return arrHilb;
  }
}
