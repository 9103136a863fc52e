/*
 * HipMODWTTransform — MODWTTransform.forwardMODWT / inverseMODWT
 * (MODWTTransform.java:256-375, DIRECT semantics) on libjwave_hip.so.
 * The flattened pow-2 API (:389-443) is inherited and calls these.
 */
package jwave.amd;

import jwave.exceptions.JWaveException;
import jwave.transforms.MODWTTransform;
import jwave.transforms.wavelets.Wavelet;

public class HipMODWTTransform extends MODWTTransform {

  private final HipNative.Taps _taps;

  public HipMODWTTransform( Wavelet wavelet ) {
    super( wavelet );
    _taps = HipNative.tapsFor( wavelet );
  }

  @Override public double[ ][ ] forwardMODWT( double[ ] data, int maxLevel ) {
    if( _taps == null || data == null || data.length == 0 )
      return super.forwardMODWT( data, maxLevel ); // reference checks + empty rows
    int n = data.length;
    if( maxLevel < 0 || !HipNative.fitsArray( maxLevel + 1, n ) )
      return super.forwardMODWT( data, maxLevel );  // reference checks, or > one Java array
    double[ ] wv = new double[ ( maxLevel + 1 ) * n ];
    try {
      HipNative.check( HipNative.modwt( HipNative.ctx( ), true, data, wv, n, maxLevel, _taps.L,
          _taps.tw, _taps.lo, _taps.hi, _taps.loR, _taps.hiR ) );
    } catch( JWaveException e ) {
      throw new IllegalStateException( e.getMessage( ), e );
    }
    return HipNative.unpack( wv, maxLevel + 1, n );
  }

  @Override public double[ ] inverseMODWT( double[ ][ ] c ) {
    if( _taps == null || c == null || c.length <= 1 )
      return super.inverseMODWT( c );
    int J = c.length - 1, n = c[ 0 ].length;
    if( !HipNative.fitsArray( J + 1, n ) )
      return super.inverseMODWT( c );
    double[ ] wv = HipNative.pack( c ), x = new double[ n ];
    try {
      HipNative.check( HipNative.modwt( HipNative.ctx( ), false, x, wv, n, J, _taps.L, _taps.tw,
          _taps.lo, _taps.hi, _taps.loR, _taps.hiR ) );
    } catch( JWaveException e ) {
      throw new IllegalStateException( e.getMessage( ), e );
    }
    return x;
  }
}
